#!/bin/bash
# Round-4 first GPU pass: full GPU suite, the parity subset on the bounds-check build (make debug), one bench line.
#   bash tools/runs/r4a.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4a}
mkdir -p $OUT
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
DBG=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_debug.so
TAGAN_LIB=$DBG timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membank.py \
    tests/test_gpu_ingest.py tests/test_gpu_temporal_v4.py tests/test_gpu_sgemm.py tests/test_gpu_debug.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/debug_tests.log 2>&1 || { tail -60 $OUT/debug_tests.log; exit 1; }
tail -1 $OUT/debug_tests.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['alt_precision']['ms_per_step'], d['roofline']['frac'], d['temporal_kernels'][1]['frac_bwd'])"
