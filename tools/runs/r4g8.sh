#!/bin/bash
# Edge-attention backward with 8 features per lane (TAGAN_GEO_FPL_BWD=8, libtagan_hip_gfpl8.so: 16-B bf16 loads per
# lane instead of 8-B) against the shipped FPL = 4, fp32 and bf16 storage, C2 and C4 graphs, two interleaved rounds.
#   bash tools/runs/r4g8.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4g8}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_gfpl8.so; do
    for cfg in c2 c4; do for dt in "" "--bf16"; do
      TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/geo_kernels.py --config $cfg --reps 10 $dt \
          > $OUT/g_${lib}_${cfg}_${rep}${dt}.json 2>&1 || { tail -5 $OUT/g_${lib}_${cfg}_${rep}${dt}.json; exit 1; }
      echo "$lib $cfg $dt $(python -c "import json;d=json.loads(open('$OUT/g_${lib}_${cfg}_${rep}${dt}.json').read().strip().splitlines()[-1]);print(d['ms_fwd'], d['ms_bwd'], d['frac'])")"
    done; done
  done
done
