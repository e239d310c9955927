#!/bin/bash
# TN A/B (k_sgemm_tn2 vs k_sgemm_tn) at H = 128 / 256 + the stream-GEMM unit tests.   bash tools/runs/r4c.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 300 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
timeout -k 10 300 python tools/tn_ab.py --H 128 > $OUT/tn_ab_h128.jsonl 2>&1 || { tail -20 $OUT/tn_ab_h128.jsonl; exit 1; }
cat $OUT/tn_ab_h128.jsonl
timeout -k 10 300 python tools/tn_ab.py --H 256 --M 1600000 > $OUT/tn_ab_h256.jsonl 2>&1 || { tail -20 $OUT/tn_ab_h256.jsonl; exit 1; }
cat $OUT/tn_ab_h256.jsonl
