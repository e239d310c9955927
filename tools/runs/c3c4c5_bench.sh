#!/bin/bash
# C3 (fp32), C4 (fp32) and C5 (bf16 activations, one GPU) bench lines on the current tree: >= 3 warm-ups, >= 5 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c345}
mkdir -p $OUT
for c in c3 c4; do
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['ms_per_step'], d['value'], d['config']['peak_hbm_gb'], d.get('breakdown'))"
done
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --precision bf16 --launch eager > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['ms_per_step'], d['value'], d['config']['peak_hbm_gb'], d.get('breakdown'))"
