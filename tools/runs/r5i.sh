#!/bin/bash
# Round 5 (i): LN1 in the QKV projection's prologue at H = 256 (32 lanes per row; libtagan_hip.so) against the
# standalone LayerNorm beside the stream GEMMs (libtagan_hip_noln256.so, TAGAN_SG_LN256=0): LN-fusion / stream-GEMM /
# geometry tests, the C3 (fp32) step on both, and the C5 bf16 step on the library GEMMs (TAGAN_SG_BF16_MAX_H=128,
# default) against the stream GEMMs (=256).   bash tools/runs/r5i.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5i}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_sgemm_ln.py tests/test_gpu_sgemm.py tests/test_gpu_fullsize.py \
    -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for lib in libtagan_hip.so libtagan_hip_noln256.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 400 python bench.py --config c3 $B > $OUT/c3_$lib.json 2> $OUT/c3_$lib.err || { tail -20 $OUT/c3_$lib.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_$lib.json'));print('c3 $lib', d['ms_per_step'], d.get('breakdown',{}).get('forward_ms'), d.get('breakdown',{}).get('backward_ms'))"
done
for mh in 128 256; do
  TAGAN_SG_BF16_MAX_H=$mh timeout -k 10 400 python bench.py --config c5 --precision bf16 $B > $OUT/c5_$mh.json 2> $OUT/c5_$mh.err || { tail -20 $OUT/c5_$mh.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_$mh.json'));print('c5 bf16 max_h=$mh', d['ms_per_step'], d.get('breakdown',{}).get('forward_ms'), d.get('breakdown',{}).get('backward_ms'))"
done
