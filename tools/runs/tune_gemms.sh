#!/bin/bash
# Tune the C2 step's GEMMs (fp32 + bf16 modes) into gpurun_out/tune/tuned.csv, then A/B the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune
mkdir -p $OUT
rm -f $OUT/tuned.csv
timeout -k 10 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --tune-gemms \
    --gemm-table $OUT/tuned.csv > $OUT/tune.json 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
wc -l $OUT/tuned.csv
for arm in tuned default tuned default; do
  if [ $arm = tuned ]; then a="--gemm-table $OUT/tuned.csv"; else a="--no-tuned-gemms"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a > $OUT/$arm.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$arm.json'));print('$arm', d['ms_per_step'], d['alt_precision']['ms_per_step'], d['config']['gemms'])"
done
