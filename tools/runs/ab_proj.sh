#!/bin/bash
# Interleaved A/B of the fused projection kernels (TAGAN_PROJ=1) against hipBLASLt + LayerNorm kernels
# (TAGAN_PROJ=0) on the default C2 bench step, 3 rounds; one JSON line per run under gpurun_out/$1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_proj}
mkdir -p $OUT
for r in 1 2 3; do
  for p in ${SETS:-all out,dc 0}; do
    TAGAN_PROJ=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/proj${p//,/_}_r$r.json 2> $OUT/proj${p//,/_}_r$r.err || { tail -5 $OUT/proj${p//,/_}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/proj${p//,/_}_r$r.json')); print('proj=$p round $r', d['ms_per_step'], 'bf16', d.get('alt_precision',{}).get('ms_per_step'))"
  done
done
