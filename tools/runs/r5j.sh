#!/bin/bash
# Round 5 (j): rocprofv3 kernel stats of the C5 bf16 step on the stream GEMMs (TAGAN_SG_BF16_MAX_H=256: LN1 prologue
# and LN2 epilogue fused at H = 256) -- which products lose to the library there (compare r5h's C5 profile).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5j}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAGAN_SG_BF16_MAX_H=256 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o run -- \
    python bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    --precision bf16 --launch eager --sub-records none > $OUT/stats_c5.log 2>&1 || { tail -20 $OUT/stats_c5.log; exit 1; }
find $OUT/stats_c5 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c5 -name "*kernel_stats.csv" | head -1) | sed -n 1,40p
