#!/bin/bash
# SQ + TCC counter passes (one rocprofv3 --pmc run each) over any command:
#   bash tools/sq_counters.sh <tag> python tools/tattn_kernels.py --config c2 --reps 2
# CSVs under gpurun_out/sq_<tag>/<first counter>/; summary: python tools/pmc_table.py gpurun_out/sq_<tag>
# (FETCH_SIZE counts wide reads at half their bytes on gfx950: double it; both are KiB.)
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" \
            "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
            "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/$name -- "$@" > $OUT/$name.log 2>&1
done
find $OUT -name "*kernel_trace*" -delete
python tools/pmc_table.py $OUT > $OUT/table.txt
