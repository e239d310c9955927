#!/bin/bash
# fp32 forward edge kernel with 4 features per lane on cache-cold batches (TAGAN_GEO_FPL_FWD_COLD=4, default) against
# 8 (libtagan_hip_cold8.so): full GPU suite on the default, geo_kernels.py C2 / C3 / C4 / C5-bf16 interleaved, the
# C4 roofline line per build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zq}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -40 $OUT/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -n 1 $OUT/gpu_tests.log)"
for r in 1 2; do
  for V in "" _cold8; do
    for C in c2 c3 c4; do
      TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python tools/geo_kernels.py --config $C --snapshots $([ $C = c2 ] && echo 32 || echo 1) > $OUT/g${V}_${C}_$r.log 2>&1 || { tail -20 $OUT/g${V}_${C}_$r.log; exit 1; }
      echo "geo $C$V run $r: $(tail -n 1 $OUT/g${V}_${C}_$r.log | python -c "import sys,json;d=json.loads(sys.stdin.read());print(d['ms_fwd'], d['ms_bwd'])")"
    done
  done
done
for V in "" _cold8; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 200 python bench.py --roofline-only --roofline-reps 10 > $OUT/roof$V.json 2> $OUT/roof$V.err || { tail -20 $OUT/roof$V.err; exit 1; }
  echo "roofline$V: $(python -c "import json;r=json.load(open('$OUT/roof$V.json'))['roofline'];print(r['frac'], r['ms_fwd'], r['ms_bwd'])")"
done
