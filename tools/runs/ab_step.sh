#!/bin/bash
# same-process interleaved A/B of the LN-fusion variants (tools/ab_step.py), fp32 and bf16, row kernel on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abs}
mkdir -p $OUT
for row in 1 0; do
  for prec in fp32 bf16; do
    TAGAN_SG_ROW=$row timeout -k 10 300 python tools/ab_step.py --precision $prec none in in+out all \
        > $OUT/ab_${row}_$prec.log 2>&1 || { tail -20 $OUT/ab_${row}_$prec.log; exit 1; }
    sed "s/^/ROW=$row /" $OUT/ab_${row}_$prec.log | grep median
  done
done
