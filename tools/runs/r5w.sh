#!/bin/bash
# Round 5 (w): LayerNorm backward with the next iteration's rows prefetched (libtagan_hip_lnpf.so, TAGAN_LN_BWD_PF=1; not kept)
# and with 4 row groups per wave (libtagan_hip_lnu4.so) against the shipped build: LN tests on the variants, the LN
# probe at C2's shape and at H = 256 (3.2M rows), the C2 step interleaved.   bash tools/runs/r5w.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5w}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for lib in libtagan_hip_lnpf.so libtagan_hip_lnu4.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_parity.py -m gpu -q \
      --timeout 300 --timeout-method thread > $OUT/tests_$lib.log 2>&1 || { tail -40 $OUT/tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/tests_$lib.log)"
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_lnpf.so libtagan_hip_lnu4.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/ln_probe.py 2>&1 | grep bwd || exit 1
    LN_PROBE_M=3200000 LN_PROBE_H=256 TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/ln_probe.py 2>&1 | grep bwd || exit 1
  done
done
for lib in libtagan_hip.so libtagan_hip_lnpf.so libtagan_hip_lnu4.so libtagan_hip.so libtagan_hip_lnpf.so libtagan_hip_lnu4.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
      > $OUT/bench_${lib}.json 2> $OUT/bench_${lib}.err || { tail -20 $OUT/bench_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${lib}.json'));print('c2 $lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
