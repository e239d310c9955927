#!/bin/bash
# CSR builder A/B over library variants: CSR tests on each, then csr_bench C2 / C4 interleaved (two rounds).
#   bash tools/runs/csr_ab.sh <tag> <variant suffix>...   (suffix "" = the default libtagan_hip.so, e.g. _rank4)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
shift
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for V in "$@"; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest.py \
      tests/test_gpu_fullsize.py -m gpu -k "csr or csc or graph or ingest" -q --timeout 200 \
      --timeout-method thread > $OUT/t$V.log 2>&1 || { tail -30 $OUT/t$V.log; exit 1; }
  echo "tests$V: $(tail -n 1 $OUT/t$V.log)"
done
for r in 1 2; do
  for V in "$@"; do
    TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python -u tools/csr_bench.py --configs c2,c4 > $OUT/b${V}_$r.log 2>&1 || { tail -30 $OUT/b${V}_$r.log; exit 1; }
    echo "bench$V run $r: $(grep build_ms $OUT/b${V}_$r.log | python -c "import sys,json;print(' '.join('%s/%d %.3f'%(d['config'],d['snapshots'],d['build_ms']) for d in map(json.loads,sys.stdin)))")"
  done
done
