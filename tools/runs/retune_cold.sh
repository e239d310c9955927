#!/bin/bash
# Re-tune the C2 step's GEMMs with TunableOp's rotating buffer (1 GB: every timed call reads operands that are not
# cache-resident, as inside the step), then interleaved A/B of the new table against the shipped one.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune3
mkdir -p $OUT
rm -f $OUT/tuned.csv
PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=1024 timeout -k 10 1000 python bench.py --steps 3 --warmup 2 --no-cpu-baseline \
    --no-roofline --no-c1 --launch eager --tune-gemms --gemm-table $OUT/tuned.csv > $OUT/tune.json 2> $OUT/tune.err \
    || { tail -20 $OUT/tune.err; exit 1; }
wc -l $OUT/tuned.csv
grep 320000 $OUT/tuned.csv
for arm in new shipped new shipped new shipped; do
  if [ $arm = new ]; then a="--gemm-table $OUT/tuned.csv"; else a=""; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-c1 $a > $OUT/$arm.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$arm.json'));print('$arm', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
