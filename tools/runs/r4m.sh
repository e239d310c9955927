#!/bin/bash
# Pair-word temporal dropout (two hashes per four elements) + keep-bit cache + pipelined v5 backward: the temporal
# GPU tests, then C5 / C3 / C2 kernel times with the keep cache on and off.   bash tools/runs/r4m.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4m}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_v4.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in c5 c3 c2; do
  for k in 1 0; do
    timeout -k 10 200 python tools/tattn_kernels.py --config $c --p 0.1 --keep $k --reps 5 > $OUT/t_${c}_$k.json 2>&1 \
        || { tail -5 $OUT/t_${c}_$k.json; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/t_${c}_$k.json').read().strip().splitlines()[-1]);print('$c keep=$k', d['keep_bits'], d['ms_fwd'], d['ms_bwd'], d['tflops_fwd'], d['tflops_bwd'], d['frac_hbm'])"
  done
done
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for c in c5 c3; do
  TAGAN_LIB=$L/libtagan_hip_noslp.so timeout -k 10 200 python tools/tattn_kernels.py --config $c --p 0.1 --keep 1 --reps 5 \
      > $OUT/t_${c}_noslp.json 2>&1 || { tail -5 $OUT/t_${c}_noslp.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/t_${c}_noslp.json').read().strip().splitlines()[-1]);print('$c noslp', d['keep_bits'], d['ms_fwd'], d['ms_bwd'], d['tflops_fwd'], d['tflops_bwd'], d['frac_hbm'])"
done
