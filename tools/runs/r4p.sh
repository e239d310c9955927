#!/bin/bash
# C3 / C4 / C5 bench lines on the round-4 tree (tools/runs/c3c4c5_bench.sh) and the C5 bf16 step with the library
# GEMMs (TAGAN_SGEMM=0) beside the hand-written ones: does the H = 256 bf16 stream-GEMM path win at C5?
#   bash tools/runs/r4p.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4p}
mkdir -p $OUT
bash tools/runs/c3c4c5_bench.sh ${1:-r4p} || exit 1
TAGAN_SGEMM=0 timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline \
    --no-alt-precision --no-c1 --precision bf16 --launch eager > $OUT/c5_lib.json 2> $OUT/c5_lib.err \
    || { tail -20 $OUT/c5_lib.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5_lib.json'));print('c5 TAGAN_SGEMM=0', d['ms_per_step'], d['value'], d.get('breakdown'))"
