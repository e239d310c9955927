#!/bin/bash
# Round 6 (i): ping-pong NT (TAGAN_SG_PP=1, libtagan_hip_pp.so) vs shipped: stream-GEMM tests on the variant, C2 fp32
# step A/B (alternating, two rounds), rocprof stream-GEMM tables of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6i}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_pppf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests_pp.log 2>&1 || { tail -30 $OUT/tests_pp.log; exit 1; }
tail -1 $OUT/tests_pp.log
for r in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_pp.so libtagan_hip_pppf.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 --no-roofline > $OUT/$lib.$r.json 2> $OUT/$lib.$r.err || { tail -20 $OUT/$lib.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$lib.$r.json'));print('$lib', $r, 'c2 fp32', d['ms_per_step'], 'bf16', d['alt_precision']['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in libtagan_hip.so libtagan_hip_pp.so libtagan_hip_pppf.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/prof_$lib.log 2>&1 || { tail -20 $OUT/prof_$lib.log; exit 1; }
  find $OUT/prof_$lib -name "*kernel_trace*" -delete
  f=$(find $OUT/prof_$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python tools/sgemm_table.py $f; python tools/kstats.py $f | sed -n 1,4p
done
