#!/bin/bash
# Round 5 (p): the bf16-storage score products (S, dP) on v_mfma_f32_16x16x16_bf16 in the v4 / v6 kernels too (C2, C4
# bf16) against libtagan_hip_nobfmm.so (TAGAN_TATTN_BFMM=0): all temporal tests, the C2 / C4 temporal kernels alone
# in bf16 storage, the C2 step (fp32 + bf16 lines) interleaved x2.   bash tools/runs/r5p.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5p}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v6.py tests/test_gpu_temporal_v5.py \
    tests/test_gpu_temporal_T.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nobfmm.so; do
    for cfg in "c2 --bf16" "c4 --bf16" "c4"; do
      TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/tattn_kernels.py --config $cfg --reps 10 > $OUT/tk.log 2>&1 || { tail -20 $OUT/tk.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/tk.log').read().strip().splitlines()[-1]);print('$lib', '$cfg', d['ms_fwd'], d['ms_bwd'])"
    done
  done
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nobfmm.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
