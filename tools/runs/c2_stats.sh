#!/bin/bash
# rocprofv3 kernel stats of the C2 bench (graph-launched steps) -> gpurun_out/$1/stats_c2; per-step summary printed.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c2s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c2 -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/stats_c2.log 2>&1 || { tail -20 $OUT/stats_c2.log; exit 1; }
find $OUT/stats_c2 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c2 -name "*kernel_stats.csv" | head -1)
