#!/bin/bash
# C2 kernel stats with the fused projection kernels on (TAGAN_PROJ=$2) vs off, one gpurun call
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pab}
mkdir -p $OUT
for P in 0 ${2:-out}; do
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  TAGAN_PROJ=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p_$P -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
      > $OUT/p_$P.log 2>&1 || { tail -20 $OUT/p_$P.log; exit 1; }
  find $OUT/p_$P -name "*kernel_trace*" -delete
  echo "== TAGAN_PROJ=$P"; grep -o '"ms_per_step": [0-9.]*' $OUT/p_$P.log
  python tools/kstats.py $(find $OUT/p_$P -name "*kernel_stats.csv" | head -1) | head -24
done
