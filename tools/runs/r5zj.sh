#!/bin/bash
# TN weight-gradient kernel: next tile's chunk loads issued during the stash (TAGAN_SG_TN_ILOAD=1, default) against
# after it (libtagan_hip_il0.so): sgemm tests, tn_ab.py at H = 128 / 256 per build, C2 fp32 / bf16 steps interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zj}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -m gpu -q --timeout 200 \
    --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
echo "sgemm tests: $(tail -n 1 $OUT/t.log)"
for V in "" _il0; do
  for H in 128 256; do
    M=$([ $H = 128 ] && echo 320000 || echo 1600000)
    TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python tools/tn_ab.py --M $M --H $H > $OUT/tn${V}_$H.log 2>&1 || { tail -20 $OUT/tn${V}_$H.log; exit 1; }
    echo "tn$V H=$H:"; cat $OUT/tn${V}_$H.log
  done
done
for r in 1 2; do
  for V in "" _il0; do
    for P in fp32 bf16; do
      TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
          --no-roofline --no-alt-precision --no-c1 --precision $P > $OUT/b${V}_${P}_$r.json 2> $OUT/b${V}_${P}_$r.err \
          || { tail -20 $OUT/b${V}_${P}_$r.err; exit 1; }
      echo "step$V $P run $r: $(python -c "import json;print(json.load(open('$OUT/b${V}_${P}_$r.json'))['ms_per_step'])")"
    done
  done
done
