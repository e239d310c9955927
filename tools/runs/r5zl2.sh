#!/bin/bash
# Edge-kernel merges (k_geo_fwd_merge, k_geo_sum_parts) with 8 / 16 partials per lane and the partial slots loaded
# ahead (default) against 4 / 4 (libtagan_hip_mg4.so, the round-4 arithmetic order): geo / graph GPU tests on the
# default and bounds-check builds, geo_kernels.py C2 per build, C2 fp32 / bf16 steps interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zl}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for V in "" _debug; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
      -m gpu -q --timeout 200 --timeout-method thread > $OUT/t$V.log 2>&1 || { tail -30 $OUT/t$V.log; exit 1; }
  echo "tests$V: $(tail -n 1 $OUT/t$V.log)"
done
for r in 1 2; do
  for V in "" _mg4; do
    TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python tools/geo_kernels.py --config c2 > $OUT/g${V}_$r.log 2>&1 || { tail -20 $OUT/g${V}_$r.log; exit 1; }
    echo "geo$V run $r: $(tail -n 2 $OUT/g${V}_$r.log | tr '\n' ' ')"
  done
done
for r in 1 2; do
  for V in "" _mg4; do
    for P in fp32 bf16; do
      TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
          --no-roofline --no-alt-precision --no-c1 --precision $P > $OUT/b${V}_${P}_$r.json 2> $OUT/b${V}_${P}_$r.err \
          || { tail -20 $OUT/b${V}_${P}_$r.err; exit 1; }
      echo "step$V $P run $r: $(python -c "import json;print(json.load(open('$OUT/b${V}_${P}_$r.json'))['ms_per_step'])")"
    done
  done
done
