#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v4g}
mkdir -p $OUT
for rep in 1 2; do
  for G in 1024 2048 4096 8192; do
    TAGAN_V4_G=$G timeout -k 10 120 python tools/tattn_kernels.py --config c2 --reps 20 > $OUT/k.json 2>$OUT/k.err || { tail -5 $OUT/k.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/k.json'));print('G=%-5s fwd %.4f bwd %.4f' % ('$G', d['ms_fwd'], d['ms_bwd']))"
  done
done
