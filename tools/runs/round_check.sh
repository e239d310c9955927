#!/bin/bash
# Full GPU test suite + default bench line + rocprof kernel stats of the bench (one gpurun call).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-chk}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats -name "*kernel_stats.csv" | head -1) 7
