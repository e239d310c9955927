#!/bin/bash
# temporal attention: v5 / T-sweep / v4 / v6 tests, then kernel times at C5, C3 and C2, into gpurun_out/<dir>
set -o pipefail
OUT=gpurun_out/${1:-tc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_T.py tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v6.py -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for c in ${2:-c5 c3 c2}; do
  timeout -k 10 300 python -u tools/tattn_kernels.py --config $c --reps 5 2>/dev/null | tee -a $OUT/k.jsonl || exit 1
done
