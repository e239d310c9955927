#!/bin/bash
# v5 backward MODE 3 with 1/(1-p) folded into the outputs and opaque keep masks (libtagan_hip.so) against the previous
# commit's build (libtagan_hip_prev.so): temporal GPU tests, then C5 / C3 / C2 kernel times interleaved x2.
#   bash tools/runs/r4o.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4o}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_v4.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for c in c5 c3; do
    for lib in libtagan_hip.so libtagan_hip_prev.so; do
      TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/tattn_kernels.py --config $c --p 0.1 --reps 5 \
          > $OUT/t_${c}_${lib}_$rep.json 2>&1 || { tail -5 $OUT/t_${c}_${lib}_$rep.json; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/t_${c}_${lib}_$rep.json').read().strip().splitlines()[-1]);print('$c $lib', d['keep_bits'], d['ms_fwd'], d['ms_bwd'], d['tflops_fwd'], d['tflops_bwd'], d['frac_hbm'])"
    done
  done
done
