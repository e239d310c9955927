#!/bin/bash
# Edge kernels at C2 (all 32 snapshots) and C4 (one snapshot) with attention dropout p = 0.1 and p = 0: what the
# per-(edge, head) dropout hash costs.   bash tools/runs/r4g2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4g2}
mkdir -p $OUT
for rep in 1 2; do
  for c in "c2 32" "c4 1"; do
    set -- $c
    for p in 0.1 0; do
      timeout -k 10 200 python tools/geo_kernels.py --config $1 --snapshots $2 --p $p --reps 20 > $OUT/g_$1_$p_$rep.json 2>&1 \
          || { tail -5 $OUT/g_$1_$p_$rep.json; exit 1; }
      echo "$1 p=$p $(tail -1 $OUT/g_$1_$p_$rep.json)"
    done
  done
done
