#!/bin/bash
# Round 5 (q): why the temporal backward is slower in bf16 storage than in fp32 (C5 v5: 53 vs 50 ms, C4 v6: 16.2 vs
# 12.2 ms) -- SQ / TCC counter passes (tools/sq_counters.sh) of the temporal kernels alone in both storage types.
#   bash tools/runs/r5q.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5q}
for cfg in c5 c4; do
  timeout -k 10 600 bash tools/sq_counters.sh ${T}_${cfg}_bf16 python tools/tattn_kernels.py --config $cfg --bf16 --reps 1 || exit 1
  timeout -k 10 600 bash tools/sq_counters.sh ${T}_${cfg}_f32 python tools/tattn_kernels.py --config $cfg --reps 1 || exit 1
  echo "== $cfg bf16"; cat gpurun_out/sq_${T}_${cfg}_bf16/table.txt
  echo "== $cfg f32"; cat gpurun_out/sq_${T}_${cfg}_f32/table.txt
done
