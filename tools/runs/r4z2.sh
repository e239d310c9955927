#!/bin/bash
# bf16 stores through the hardware conversion (v_cvt_pk_bf16_f32) instead of the integer RNE sequence
# (libtagan_hip.so) vs the previous commit (libtagan_hip_prev.so): the bf16 GPU tests on the new build, then the C2
# step (fp32, bf16) interleaved x3 and the bf16 kernel stats of both.   bash tools/runs/r4z2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4z2}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py \
    tests/test_gpu_layernorm.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2 3; do
  for lib in libtagan_hip.so libtagan_hip_prev.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
