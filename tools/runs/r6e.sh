#!/bin/bash
# Round 6 (e): A/B of the library built without packed-FP32 VALU instructions (make variant NAME=nopk
# EXTRA="-Xclang -target-feature -Xclang -packed-fp32-ops") against the shipped build: C2 step fp32 / bf16, the C4
# edge-kernel roofline group and the temporal kernels (bench.py's own line), alternating builds, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6e}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for r in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nopk.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 > $OUT/$lib.$r.json 2> $OUT/$lib.$r.err || { tail -20 $OUT/$lib.$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$OUT/$lib.$r.json'));R=d['roofline'];T=d['temporal_kernels']
print('$lib', $r, 'c2 fp32', d['ms_per_step'], 'bf16', d['alt_precision']['ms_per_step'], 'c4 geo fwd/bwd', R.get('ms_fwd'), R.get('ms_bwd'), 'frac', R['frac'], 'tattn', [(t.get('config'), t.get('ms_fwd'), t.get('ms_bwd')) for t in T])"
  done
done
