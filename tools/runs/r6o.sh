#!/bin/bash
# Round 6 (o): H = 256 one-plane LN2 backward + out-projection gradients in one pass (k_ln2_bwd_out256): its tests,
# the full-size / bf16 tests, C5 bf16 A/B against the build without it, kernel stats of the new build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6o}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_sgemm_ln.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_noln256.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --precision bf16 > $OUT/c5_$lib.$r.json 2> $OUT/c5_$lib.$r.err || { tail -20 $OUT/c5_$lib.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c5_$lib.$r.json'));print('c5 bf16 $lib $r', d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- \
    python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --precision bf16 \
    > $OUT/c5p.json 2> $OUT/c5p.err || { tail -20 $OUT/c5p.err; exit 1; }
find $OUT/prof_c5 -name "*kernel_trace*" -delete
f=$(find $OUT/prof_c5 -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f | sed -n 1,24p
