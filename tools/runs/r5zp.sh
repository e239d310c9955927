#!/bin/bash
# Edge-kernel features per lane on the round-5 block order: fp32 backward FPL 8 (shipped 4), forward FPL 4 (shipped 8):
# geo tests on each variant, geo_kernels.py C2 / C4 interleaved, C2 fp32 step per build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zp}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for V in _fplb8 _fplf4; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "geo or metric or order" \
      --timeout 200 --timeout-method thread > $OUT/t$V.log 2>&1 || { tail -30 $OUT/t$V.log; exit 1; }
  echo "tests$V: $(tail -n 1 $OUT/t$V.log)"
done
for r in 1 2; do
  for V in "" _fplb8 _fplf4; do
    for C in c2 c4; do
      TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python tools/geo_kernels.py --config $C --snapshots $([ $C = c2 ] && echo 32 || echo 1) > $OUT/g${V}_${C}_$r.log 2>&1 || { tail -20 $OUT/g${V}_${C}_$r.log; exit 1; }
      echo "geo $C$V run $r: $(tail -n 1 $OUT/g${V}_${C}_$r.log | python -c "import sys,json;d=json.loads(sys.stdin.read());print(d['ms_fwd'], d['ms_bwd'])")"
    done
  done
done
for V in "" _fplb8 _fplf4; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-roofline --no-alt-precision --no-c1 > $OUT/b$V.json 2> $OUT/b$V.err || { tail -20 $OUT/b$V.err; exit 1; }
  echo "step$V: $(python -c "import json;print(json.load(open('$OUT/b$V.json'))['ms_per_step'])")"
done
