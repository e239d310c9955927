#!/bin/bash
# Grid-size sweep of the v4 temporal kernels (TAGAN_V4_G row groups x heads waves), C2 and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v4g
mkdir -p $OUT
for rep in 1 2; do
  for G in 256 384 512 640 768 1024; do
    for cfg in c2 c4; do
      TAGAN_V4_G=$G timeout -k 10 120 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('$OUT/k.json'));print('G=%-5s %s fwd %.4f bwd %.4f' % ('$G', '$cfg', d['ms_fwd'], d['ms_bwd']))"
    done
  done
done
