#!/bin/bash
# Round 6 (ah): merge accumulator defaults in the whole step: (sum 16, fwd 8) shipped vs (16, 16) vs (8, 8), ABAB.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6ah}
mkdir -p $OUT
for r in 1 2; do
  for v in "16 8" "16 16" "8 8"; do
    set -- $v
    TAGAN_GEO_MG=$1 TAGAN_GEO_MG_FWD=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 --no-roofline > $OUT/b_$1_$2.$r.json 2> $OUT/b_$1_$2.$r.err || { tail -20 $OUT/b_$1_$2.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_$1_$2.$r.json'));print('sum $1 fwd $2 run $r c2', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
