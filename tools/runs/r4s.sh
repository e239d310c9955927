#!/bin/bash
# Geometric merge kernels with more partial loads in flight (forward merge 8 states, partial sums 16 accumulators per
# lane): the geometric / parity GPU tests, then kernel stats of the C2 step.   bash tools/runs/r4s.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_debug.py tests/test_gpu_fullsize.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c2 -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/stats_c2.log 2>&1 || { tail -20 $OUT/stats_c2.log; exit 1; }
find $OUT/stats_c2 -name "*kernel_trace*" -delete
f=$(find $OUT/stats_c2 -name "*kernel_stats.csv" | head -1)
grep "k_geo_sum_parts\|k_geo_fwd_merge" $f | cut -d, -f1-4
python tools/kstats.py $f | sed -n 1,6p
