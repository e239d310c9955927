#!/bin/bash
# Round 6 (n): fused skip-LayerNorm backward at H = 256: LayerNorm / full-size tests, C3 fp32 and C5 bf16 step lines
# with their kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c3 c5; do
  P=fp32; [ $c = c5 ] && P=bf16
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- \
    python bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --precision $P \
    > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
  find $OUT/prof_$c -name "*kernel_trace*" -delete
  f=$(find $OUT/prof_$c -name "*kernel_stats.csv" | head -1)
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['ms_per_step'], '(profiled)')"
  python tools/kstats.py $f | sed -n 1,8p
done
for c in c3 c5; do
  P=fp32; [ $c = c5 ] && P=bf16
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --precision $P > $OUT/${c}_clean.json 2> $OUT/${c}_clean.err || { tail -20 $OUT/${c}_clean.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}_clean.json'));print('$c clean', d['ms_per_step'])"
done
