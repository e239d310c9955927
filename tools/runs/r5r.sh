#!/bin/bash
# Round 5 (r): temporal v5 / v6 kernels with the prefetched rows kept in their stored form until use (bf16 storage: no
# conversion at the load, so the prefetch no longer waits there) against the previous commit (libtagan_hip_prev.so):
# all temporal tests, the C5 / C4 temporal kernels alone (bf16, fp32), the C5 bf16 step and the C2 step, interleaved.
#   bash tools/runs/r5r.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5r}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v6.py tests/test_gpu_temporal_v5.py \
    tests/test_gpu_temporal_T.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_prev.so; do
    for cfg in "c5 --bf16" "c4 --bf16" "c5" "c4"; do
      TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/tattn_kernels.py --config $cfg --reps 10 > $OUT/tk.log 2>&1 || { tail -20 $OUT/tk.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/tk.log').read().strip().splitlines()[-1]);print('$lib', '$cfg', d['ms_fwd'], d['ms_bwd'])"
    done
  done
done
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for lib in libtagan_hip.so libtagan_hip_prev.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 400 python bench.py --config c5 --precision bf16 $B > $OUT/c5_${lib}.json 2> $OUT/c5_${lib}.err || { tail -20 $OUT/c5_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_${lib}.json'));print('c5 bf16 $lib', d['ms_per_step'])"
done
for lib in libtagan_hip.so libtagan_hip_prev.so libtagan_hip.so libtagan_hip_prev.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
      > $OUT/bench_${lib}.json 2> $OUT/bench_${lib}.err || { tail -20 $OUT/bench_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${lib}.json'));print('c2 $lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
