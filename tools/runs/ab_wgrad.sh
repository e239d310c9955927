#!/bin/bash
# Interleaved A/B of the QKV weight-gradient slice height (8192 -> 8000 at C2, vs 2048 -> 2560), tuned table.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/abw
mkdir -p $OUT
cp temporal-asymmetric-graph-attention-network_amd/tuned_gemms_gfx950.csv $OUT/tuned.csv
TAGAN_WGRAD_ROWS_QKV=8192 timeout -k 10 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --tune-gemms \
    --gemm-table $OUT/tuned.csv > /dev/null 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
for rep in 1 2 3; do
  for r in 8192 2048; do
    TAGAN_WGRAD_ROWS_QKV=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --gemm-table $OUT/tuned.csv > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b.json'));print('rows=$r', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
