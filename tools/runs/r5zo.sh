#!/bin/bash
# v4 temporal backward occupancy bound (TAGAN_V4_WPE_B: shipped 3 against 2 and 4): C2 / C4-bf16 kernel timings
# interleaved, then the C2 fp32 step per build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zo}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for r in 1 2; do
  for V in "" _wpeb2 _wpeb4; do
    TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python tools/tattn_kernels.py --config c2 > $OUT/k${V}_$r.log 2>&1 || { tail -20 $OUT/k${V}_$r.log; exit 1; }
    echo "tattn c2$V run $r: $(tail -n 1 $OUT/k${V}_$r.log)"
  done
done
for V in "" _wpeb2 _wpeb4; do
  TAGAN_LIB=$L/libtagan_hip$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-roofline --no-alt-precision --no-c1 > $OUT/b$V.json 2> $OUT/b$V.err || { tail -20 $OUT/b$V.err; exit 1; }
  echo "step$V: $(python -c "import json;print(json.load(open('$OUT/b$V.json'))['ms_per_step'])")"
done
