#!/bin/bash
# matrix-core / VALU overlap counters over a command: bash tools/runs/mfma_pmc.sh <tag> <cmd...>
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/mp_$TAG
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/p1 -- "$@" > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
find $OUT -name "*kernel_trace*" -delete
python tools/pmc_table.py $OUT tattn
