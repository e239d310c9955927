#!/bin/bash
# Add the C1 step's GEMM shapes to the shipped TunableOp table, then A/B the C1 line (graph launch) new vs shipped.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune_c1
mkdir -p $OUT
cp temporal-asymmetric-graph-attention-network_amd/tuned_gemms_gfx950.csv $OUT/table.csv
timeout -k 10 600 python bench.py --config c1 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --launch eager \
    --tune-gemms --gemm-table $OUT/table.csv > $OUT/tune.json 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
wc -l $OUT/table.csv
for arm in new shipped new shipped; do
  if [ $arm = new ]; then a="--gemm-table $OUT/table.csv"; else a=""; fi
  timeout -k 10 200 python bench.py --config c1 --steps 50 --warmup 10 --no-cpu-baseline --no-roofline --launch graph $a > $OUT/$arm.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$arm.json'));print('$arm', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --gemm-table $OUT/table.csv > $OUT/c2.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$OUT/c2.json'));print('c2 with new table', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
