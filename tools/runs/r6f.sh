#!/bin/bash
# Round 6 (f): per-kernel C2 bf16-step stats of the shipped and packed-FP32-free (nopk) builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in libtagan_hip.so libtagan_hip_nopk.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --precision bf16 \
    > $OUT/$lib.log 2>&1 || { tail -20 $OUT/$lib.log; exit 1; }
  find $OUT/$lib -name "*kernel_trace*" -delete
done
