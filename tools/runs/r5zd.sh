#!/bin/bash
# Round 5 (zd): the H = 256 one-plane QKV projection with the LN1 prologue over two column groups of three n-subtiles
# per wave (libtagan_hip_ln256w.so, TAGAN_SG_LN256_WIDE=1: x read twice instead of three times) against three groups
# of two: stream-GEMM / LN tests on the variant, the H = 256 bf16 probe, the C5 bf16 step interleaved x2.
#   bash tools/runs/r5zd.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zd}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_ln256w.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -m gpu -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libtagan_hip.so libtagan_hip_ln256w.so libtagan_hip.so libtagan_hip_ln256w.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/sgemm_probe.py --H 256 --M 3200000 --planes 1 --cases qkv_fwd_ln \
      > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
  python -c "
import json
for l in open('$OUT/probe.log'):
    if l.startswith('{'):
        c = json.loads(l); print('$lib', '%-22s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
done
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for lib in libtagan_hip.so libtagan_hip_ln256w.so libtagan_hip.so libtagan_hip_ln256w.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 500 python bench.py --config c5 --precision bf16 $B > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5 $lib', d['ms_per_step'])"
done
