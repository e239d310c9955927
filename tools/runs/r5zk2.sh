#!/bin/bash
# Round-5 final tree: two more default C2 bench lines (box spread) and the C3 / C4 / C5 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zk}_c345
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --no-c1 > $OUT/c2_$r.json 2> $OUT/c2_$r.err || { tail -20 $OUT/c2_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_$r.json'));print('c2 run $r', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
bash tools/runs/c3c4c5_bench.sh ${1:-r5zk}_c345 || exit 1
