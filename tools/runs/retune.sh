#!/bin/bash
# Full GPU suite, then re-tune the GEMM table from the shipped one (adds new shapes), then bench twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/retune
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
cp temporal-asymmetric-graph-attention-network_amd/tuned_gemms_gfx950.csv $OUT/tuned.csv
timeout -k 10 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --tune-gemms \
    --gemm-table $OUT/tuned.csv > $OUT/tune.json 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
wc -l $OUT/tuned.csv
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --gemm-table $OUT/tuned.csv > $OUT/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/b.json'));print(d['ms_per_step'], d['alt_precision']['ms_per_step'], d['breakdown'])"
done
