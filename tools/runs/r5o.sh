#!/bin/bash
# Round 5 (o): the bf16-storage temporal v5 kernels with the score products S = K.Q^T and dP = V.dO^T on
# v_mfma_f32_16x16x16_bf16 (stored bf16 operands: the same products, fp32 accumulation) against every product on
# v_mfma_f32_16x16x4_f32 (libtagan_hip_nobfmm.so, TAGAN_TATTN_BFMM=0): temporal tests on the new default, the C5 / C3
# temporal kernels alone (bf16 and fp32 storage), then the C5 bf16 step interleaved x2.   bash tools/runs/r5o.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5o}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_temporal_v5.py tests/test_gpu_temporal_T.py -m gpu -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nobfmm.so; do
    for cfg in "c5 --bf16" "c3 --bf16" "c5"; do
      TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/tattn_kernels.py --config $cfg --reps 10 > $OUT/tk.log 2>&1 || { tail -20 $OUT/tk.log; exit 1; }
      echo "$lib $cfg: $(tail -1 $OUT/tk.log)"
    done
  done
done
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nobfmm.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 400 python bench.py --config c5 --precision bf16 $B > $OUT/c5_${lib}_$rep.json 2> $OUT/c5_${lib}_$rep.err || { tail -20 $OUT/c5_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c5_${lib}_$rep.json'));print('c5 bf16 $lib', d['ms_per_step'], d.get('breakdown',{}).get('forward_ms'), d.get('breakdown',{}).get('backward_ms'))"
  done
done
