#!/bin/bash
# bf16 QKV weight gradient over three column groups at 4 waves / SIMD (libtagan_hip_tng3.so) vs the shipped one-group
# kernel: stream-GEMM GPU tests on the variant, then the C2 bf16 step (alt_precision) interleaved x3.
#   bash tools/runs/r4w.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4w}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_tng3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2 3; do
  for lib in libtagan_hip.so libtagan_hip_tng3.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
