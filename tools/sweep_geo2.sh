#!/bin/bash
# Second edge-kernel sweep + SQ/TCC counters (run through gpurun).
set -e
mkdir -p gpurun_out/sweep2
OUT=gpurun_out/sweep2/geo.jsonl
run() { timeout -k 10 300 python tools/geo_kernels.py "$@" >> $OUT 2>> gpurun_out/sweep2/geo.err; }
run --config c2
run --config c2 --chunk 64
TAGAN_LIB=variants/libtagan_u1.so run --config c2
TAGAN_LIB=variants/libtagan_u4.so run --config c2
run --config c2 --p 0
run --config c2 --metric 6 --p 0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/sweep2/sq -- python tools/geo_kernels.py --config c2 --reps 2 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/sweep2/tcc -- python tools/geo_kernels.py --config c2 --reps 2 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/sweep2/sq2 -- python tools/geo_kernels.py --config c2 --reps 2 > /dev/null 2>&1 || echo "sq2 pass failed"
