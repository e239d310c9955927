#!/bin/bash
# Interleaved A/B of an environment switch on the C2 bench (same box): bash tools/runs/ab_env.sh VAR [table]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab
mkdir -p $OUT
T=${2:+--gemm-table $2}
for rep in 1 2 3; do
  for v in 1 0; do
    env $1=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $T > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$1=$v', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
