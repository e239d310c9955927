#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rcc}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_graph.py tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py -q --timeout 300 \
    --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
