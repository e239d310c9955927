#!/bin/bash
# Geometric merge / partial-sum grid cap 4096 workgroups (shipped) vs 1024 (libtagan_hip_mg1k.so): C2 kernel stats of
# both, interleaved x2.   bash tools/runs/r4t.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4t}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_mg1k.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s_${lib}_$rep -o run -- \
        python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
        > $OUT/s_${lib}_$rep.log 2>&1 || { tail -20 $OUT/s_${lib}_$rep.log; exit 1; }
    find $OUT/s_${lib}_$rep -name "*kernel_trace*" -delete
    f=$(find $OUT/s_${lib}_$rep -name "*kernel_stats.csv" | head -1)
    echo "== $lib $rep"; grep "k_geo_sum_parts\|k_geo_fwd_merge" $f | cut -d, -f2-4
  done
done
