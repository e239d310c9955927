#!/bin/bash
# Round-end rehearsal: full GPU suite without -x (parity maxima logged), the parity subset on the bounds-check build
# (libtagan_hip_debug.so, make debug), smoke(), default bench line, rocprof kernel stats of the C2 fp32 step, the
# stream-GEMM table.  bash tools/runs/round_end.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rend}
mkdir -p $OUT
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
TAGAN_LIB=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_debug.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membank.py tests/test_gpu_ingest.py \
    tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_v6.py tests/test_gpu_sgemm.py \
    tests/test_gpu_sgemm_ln.py tests/test_gpu_debug.py tests/test_gpu_head.py tests/test_gpu_narrow.py \
    tests/test_gpu_bias_table.py -m gpu \
    -q --timeout 300 --timeout-method thread > $OUT/debug_tests.log 2>&1 || { tail -40 $OUT/debug_tests.log; exit 1; }
tail -1 $OUT/debug_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['alt_precision']['ms_per_step'], d['roofline']['frac'], d['temporal_kernels'][1]['frac_bwd'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c2 -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/stats_c2.log 2>&1 || { tail -20 $OUT/stats_c2.log; exit 1; }
find $OUT/stats_c2 -name "*kernel_trace*" -delete
f=$(find $OUT/stats_c2 -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f | sed -n 1,14p
python tools/sgemm_table.py $f
