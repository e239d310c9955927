#!/bin/bash
# Round 5 (q): why the C5 temporal backward is slower in bf16 storage than in fp32 -- SQ / TCC counter passes
# (tools/sq_counters.sh) of the C5 temporal kernels alone in both storage types.   bash tools/runs/r5q.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5q}
mkdir -p $OUT
bash tools/sq_counters.sh ${1:-r5q}_bf16 python tools/tattn_kernels.py --config c5 --bf16 --reps 1 || exit 1
bash tools/sq_counters.sh ${1:-r5q}_f32 python tools/tattn_kernels.py --config c5 --reps 1 || exit 1
echo "== bf16"; cat gpurun_out/sq_${1:-r5q}_bf16/table.txt
echo "== f32"; cat gpurun_out/sq_${1:-r5q}_f32/table.txt
