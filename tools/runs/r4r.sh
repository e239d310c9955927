#!/bin/bash
# In-step A/B of the LayerNorm launch shape (C2 bench, fp32 and bf16): the shipped library (2 row groups per wave,
# 1024 backward blocks) against 4 row groups (lnu4), 2048 blocks (lnb2k), 512 blocks (lnb512); interleaved x2.
#   bash tools/runs/r4r.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4r}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_lnu4.so libtagan_hip_lnb2k.so libtagan_hip_lnb512.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
