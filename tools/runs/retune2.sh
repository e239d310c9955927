#!/bin/bash
# Re-tune the C2 step's GEMMs on the current tree into gpurun_out/tune2/tuned.csv, then A/B new table vs shipped.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune2
mkdir -p $OUT
rm -f $OUT/tuned.csv
timeout -k 10 900 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --launch eager --tune-gemms \
    --gemm-table $OUT/tuned.csv > $OUT/tune.json 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
wc -l $OUT/tuned.csv
for arm in new shipped new shipped; do
  if [ $arm = new ]; then a="--gemm-table $OUT/tuned.csv"; else a=""; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a > $OUT/$arm.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$arm.json'));print('$arm', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
