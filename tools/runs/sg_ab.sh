#!/bin/bash
# stream-GEMM unit tests, then an interleaved C2 A/B over "ENV=VAL[,ENV=VAL]" variants (space-separated; "base" =
# no override).  bash tools/runs/sg_ab.sh <tag> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sgab}
shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 120 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
for r in 1 2; do
  for v in "$@"; do
    envs=""
    [ "$v" != "base" ] && envs=$(echo "$v" | tr ',' ' ')
    tag=$(echo "$v" | tr ',=' '_-')
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/b_${tag}_$r.json 2> $OUT/b_${tag}_$r.err || { tail -20 $OUT/b_${tag}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${tag}_$r.json'));print('$v', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
