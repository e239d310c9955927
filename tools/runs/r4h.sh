#!/bin/bash
# C3 / C4 / C5 bench lines (tools/runs/c3c4c5_bench.sh) + rocprofv3 kernel stats of 3 C3 steps (which GEMM kernels
# the H = 256 attention blocks run).   bash tools/runs/r4h.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4h}
mkdir -p $OUT
bash tools/runs/c3c4c5_bench.sh ${1:-r4h} || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c3 -o run -- \
    python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    --launch eager > $OUT/stats_c3.log 2>&1 || { tail -20 $OUT/stats_c3.log; exit 1; }
find $OUT/stats_c3 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c3 -name "*kernel_stats.csv" | head -1) | sed -n 1,24p
