#!/bin/bash
# Per-tile global reservation in the staged CSR partition passes (TAGAN_CSR_TILE_RES=1, default: no histogram pre-pass
# re-reading each block's chunk) against the block pre-pass (libtagan_hip_tres0.so): CSR tests on both (and the
# bounds-check build), csr_bench C2 / C4 interleaved, kernel stats of the C4 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zf}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for V in "" _tres0 _debug; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest.py \
      tests/test_gpu_fullsize.py -m gpu -k "csr or csc or graph or ingest" -q --timeout 200 \
      --timeout-method thread > $OUT/t$V.log 2>&1 || { tail -30 $OUT/t$V.log; exit 1; }
  echo "tests$V: $(tail -1 $OUT/t$V.log)"
done
for r in 1 2; do
  for V in "" _tres0; do
    TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python -u tools/csr_bench.py --configs c2,c4 > $OUT/b${V}_$r.log 2>&1 || { tail -30 $OUT/b${V}_$r.log; exit 1; }
    echo "bench$V run $r:"; grep build_ms $OUT/b${V}_$r.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python tools/csr_bench.py --configs c4 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_trace*" -delete
f=$(find $OUT/stats -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s %6s %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
