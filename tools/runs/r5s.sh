#!/bin/bash
# Round 5 (s): the v4 kernels (C2 backward) with their prefetched rows kept in stored form until use, against the
# build with that change in v5 / v6 only (libtagan_hip_prev.so): all temporal tests, the C2 temporal kernels alone
# (bf16, fp32), the C2 step interleaved x2.   bash tools/runs/r5s.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5s}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v6.py tests/test_gpu_temporal_v5.py \
    tests/test_gpu_temporal_T.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_prev.so; do
    for cfg in "c2 --bf16" "c2"; do
      TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/tk.log 2>&1 || { tail -20 $OUT/tk.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/tk.log').read().strip().splitlines()[-1]);print('$lib', '$cfg', d['ms_fwd'], d['ms_bwd'])"
    done
  done
done
for lib in libtagan_hip.so libtagan_hip_prev.so libtagan_hip.so libtagan_hip_prev.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
      > $OUT/bench_${lib}.json 2> $OUT/bench_${lib}.err || { tail -20 $OUT/bench_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${lib}.json'));print('c2 $lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
