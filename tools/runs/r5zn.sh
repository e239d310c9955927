#!/bin/bash
# rocprofv3 kernel stats of the C5 bf16 step on the final round-5 tree (3 profiled eager steps after 2 warm-ups).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zn}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o run -- \
    python bench.py --config c5 --precision bf16 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline \
    --no-alt-precision --no-c1 --launch eager > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
find $OUT/stats_c5 -name "*kernel_trace*" -delete
f=$(find $OUT/stats_c5 -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f 5 | sed -n 1,30p
