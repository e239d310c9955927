#!/bin/bash
# Round 5 (x): rocprofv3 kernel stats of the C5 (bf16), C3 and C4 (fp32) steps after the edge-kernel block order and the bf16 temporal changes, eager, 2 + 3 steps:
# where those configs' time goes (temporal, edge, GEMM, LayerNorm shares).   bash tools/runs/r5x.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c5 c3 c4; do
  P=fp32; [ $c = c5 ] && P=bf16
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$c -o run -- \
      python bench.py --config $c --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
      --precision $P --launch eager --sub-records none > $OUT/stats_$c.log 2>&1 || { tail -20 $OUT/stats_$c.log; exit 1; }
  find $OUT/stats_$c -name "*kernel_trace*" -delete
  echo "== $c"; python tools/kstats.py $(find $OUT/stats_$c -name "*kernel_stats.csv" | head -1) | sed -n 1,30p
done
