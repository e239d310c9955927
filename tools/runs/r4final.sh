#!/bin/bash
# Final round-4 rehearsal: tools/runs/round_end.sh (GPU suite, smoke, bench, C2 kernel stats, stream-GEMM table) and the
# parity subset on the bounds-check build.   bash tools/runs/r4final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/runs/round_end.sh ${1:-r4final} || exit 1
OUT=gpurun_out/${1:-r4final}
TAGAN_LIB=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_debug.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membank.py tests/test_gpu_ingest.py \
    tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py tests/test_gpu_sgemm.py tests/test_gpu_debug.py -m gpu \
    -x -q --timeout 300 --timeout-method thread > $OUT/debug_tests.log 2>&1 || { tail -40 $OUT/debug_tests.log; exit 1; }
tail -1 $OUT/debug_tests.log
