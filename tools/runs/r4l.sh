#!/bin/bash
# v5 temporal kernels with the dropout keep-bit cache and the software-pipelined backward phase 1: the v4/v5 temporal
# GPU tests, then C5 / C3 kernel times: keep bits on / off, pipelined (shipped) vs libtagan_hip_il0.so, p = 0.
#   bash tools/runs/r4l.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4l}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_v4.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in c5 c3; do
  for v in "libtagan_hip.so 0.1 1" "libtagan_hip.so 0.1 0" "libtagan_hip_il0.so 0.1 1" "libtagan_hip.so 0 1"; do
    set -- $v
    TAGAN_LIB=$L/$1 timeout -k 10 200 python tools/tattn_kernels.py --config $c --p $2 --keep $3 --reps 5 \
        > $OUT/t_${c}_$1_$2_$3.json 2>&1 || { tail -5 $OUT/t_${c}_$1_$2_$3.json; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/t_${c}_$1_$2_$3.json').read().strip().splitlines()[-1]);print('$c $1 p=$2 keep=$3', d['keep_bits'], d['ms_fwd'], d['ms_bwd'], d['tflops_fwd'], d['tflops_bwd'])"
  done
done
