#!/bin/bash
# C2 temporal backward: v4 (default) vs the v6 head-group slab kernel forced (TAGAN_TATTN_V6=2) at GH = 2 / 4 / 8
# heads per workgroup, interleaved x2.   bash tools/runs/r4q.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4q}
mkdir -p $OUT
for rep in 1 2; do
  for v in "1 4" "2 2" "2 4" "2 8"; do
    set -- $v
    TAGAN_TATTN_V6=$1 TAGAN_V6_GH=$2 timeout -k 10 200 python tools/tattn_kernels.py --config c2 --p 0.1 --reps 20 \
        > $OUT/t_$1_$2_$rep.json 2>&1 || { tail -5 $OUT/t_$1_$2_$rep.json; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/t_$1_$2_$rep.json').read().strip().splitlines()[-1]);print('V6=$1 GH=$2', d['ms_fwd'], d['ms_bwd'], d['gbs_fwd'], d['gbs_bwd'])"
  done
done
