#!/bin/bash
# Round 5 (zb): H = 256 three-plane weight gradients (TN) with two n-subtiles per wave (libtagan_hip_tn256.so,
# TAGAN_SG_TN256N2=1: half the column groups re-reading X, 12 MFMAs per X fragment read) against one n-subtile:
# stream-GEMM tests on the variant, the H = 256 probe, the C3 step interleaved.   bash tools/runs/r5zb.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zb}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_tn256.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -m gpu -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libtagan_hip.so libtagan_hip_tn256.so libtagan_hip.so libtagan_hip_tn256.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/sgemm_probe.py --H 256 --M 1600000 --planes 3 --cases dw_qkv,dw_o \
      > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
  python -c "
import json
for l in open('$OUT/probe.log'):
    if l.startswith('{'):
        c = json.loads(l); print('$lib', '%-22s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
done
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for lib in libtagan_hip.so libtagan_hip_tn256.so libtagan_hip.so libtagan_hip_tn256.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 500 python bench.py --config c3 $B > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3.json'));print('c3 $lib', d['ms_per_step'])"
done
