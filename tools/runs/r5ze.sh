#!/bin/bash
# Round 5 (ze): the one-plane H = 256 QKV input gradient (K = 768, N = 256, bf16 dqkv) over one workgroup column of
# two n-subtiles per wave (libtagan_hip_dh256w.so, TAGAN_SG_DH256_WIDE=1: dqkv read once instead of by two column
# groups) against two columns of one: stream-GEMM tests on the variant, the C5 bf16 step interleaved x2.
#   bash tools/runs/r5ze.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5ze}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_dh256w.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -m gpu -q \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for lib in libtagan_hip.so libtagan_hip_dh256w.so libtagan_hip.so libtagan_hip_dh256w.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 500 python bench.py --config c5 --precision bf16 $B > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5 $lib', d['ms_per_step'])"
done
