#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rlc}
mkdir -p $OUT
TAGAN_SG_ROW=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py tests/test_gpu_bf16.py -x -q \
    --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for r in 1 2; do
  for lv in 1 3; do
    TAGAN_SG_ROW=$lv timeout -k 10 300 python tools/ab_step.py --precision bf16 --rounds 5 auto > $OUT/ab_${lv}_$r.log 2>&1 \
        || { tail -20 $OUT/ab_${lv}_$r.log; exit 1; }
    echo "ROW=$lv $(grep median $OUT/ab_${lv}_$r.log)"
  done
done
