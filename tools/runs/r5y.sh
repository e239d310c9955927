#!/bin/bash
# Round 5 (y): CSR / CSC finish and place kernels with their global loads batched (kept; 1024-entry buckets not kept) (8 in flight per thread instead of
# one load -> LDS store chain) against the previous commit (libtagan_hip_prev.so), and with 1024-entry buckets on top
# (libtagan_hip_csr1k.so, TAGAN_CSR_TARGET=1024): CSR tests, csr_bench C2 / C4 interleaved x2.   bash tools/runs/r5y.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5y}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for lib in libtagan_hip.so libtagan_hip_csr1k.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -k "csr or csc" \
      --timeout 300 --timeout-method thread > $OUT/tests_$lib.log 2>&1 || { tail -40 $OUT/tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/tests_$lib.log)"
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_prev.so libtagan_hip_csr1k.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/csr_bench.py --configs c2,c4 --reps 10 --out $OUT/csr_${lib}_$rep.json > $OUT/cb.log 2>&1 || { tail -20 $OUT/cb.log; exit 1; }
    python -c "
import json
for r in json.load(open('$OUT/csr_${lib}_$rep.json')): print('$lib', r['config'], r['snapshots'], r['build_ms'])"
  done
done
