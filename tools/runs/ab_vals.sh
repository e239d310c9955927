#!/bin/bash
# Interleaved A/B of one environment variable's values on the C2 bench (same box):
#   bash tools/runs/ab_vals.sh VAR VALUE_A VALUE_B [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab
mkdir -p $OUT
VAR=$1; A=$2; B=$3; shift 3
for rep in 1 2 3; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-c1 "$@" > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$VAR=$v', d['ms_per_step'], d['alt_precision']['ms_per_step'], d['breakdown']['backward_ms'])"
  done
done
