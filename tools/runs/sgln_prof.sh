#!/bin/bash
# rocprofv3 kernel stats of the C2 step, fp32 and bf16, with the LN-fused GEMMs (TAGAN_SG_LN=1) and without.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sglnp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0; do
  for prec in fp32 bf16; do
    TAGAN_SG_LN=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s_${v}_$prec -o run -- \
      python bench.py --steps 20 --warmup 3 --precision $prec --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
      > $OUT/s_${v}_$prec.log 2>&1 || { tail -20 $OUT/s_${v}_$prec.log; exit 1; }
    find $OUT/s_${v}_$prec -name "*kernel_trace*" -delete
    echo "== SG_LN=$v $prec"
    python tools/kstats.py $(find $OUT/s_${v}_$prec -name "*kernel_stats.csv" | head -1) | sed -n 1,24p
  done
done
