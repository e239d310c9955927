#!/bin/bash
# stream-GEMM unit tests + the C2 bench line + fp32/bf16 kernel stats (tools/runs/c2_prof2.sh).  <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sgq}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 120 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
bash tools/runs/c2_prof2.sh $1
