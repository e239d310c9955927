#!/bin/bash
# TunableOp A/B for the C2 bench's GEMMs: tune once (results CSV under gpurun_out/tunable/), then
# bench with the tuned table vs without.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tunable
mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/base.json 2>$OUT/base.err || exit 1
echo "base $(python -c "import json;d=json.load(open('$OUT/base.json'));print(d['ms_per_step'])")"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tuned%d.csv \
  timeout -k 10 500 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/tune.json 2>$OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
ls -la $OUT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tuned%d.csv \
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/tuned.json 2>$OUT/tuned.err || exit 1
echo "tuned $(python -c "import json;d=json.load(open('$OUT/tuned.json'));print(d['ms_per_step'])")"
