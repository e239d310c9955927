#!/bin/bash
# SQ / TCC counters of the edge kernels at C2 (run through gpurun); CSVs under gpurun_out/geoc/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/geoc
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/geoc/$name -- \
      python tools/geo_kernels.py --config c2 --reps 2 > gpurun_out/geoc/$name.log 2>&1 || echo "pass $name failed"
done
find gpurun_out/geoc -name "*kernel_trace*" -delete
