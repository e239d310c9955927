#!/bin/bash
# The graph-capture tests (incl. the T = 128 keep-bit cache under capture).   bash tools/runs/r4y.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4y}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -10
