#!/bin/bash
# C4 edge-kernel roofline line: the shipped library against the build of commit 2aafa4a (libtagan_hip_r4old.so, before
# the DPP lane-reduction change), interleaved x3 on one box.   bash tools/runs/r4u.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4u}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for rep in 1 2 3; do
  for lib in libtagan_hip.so libtagan_hip_r4old.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 200 python bench.py --roofline-only --roofline-reps 10 > $OUT/roof_${lib}_$rep.json \
        2> $OUT/roof_${lib}_$rep.err || { tail -20 $OUT/roof_${lib}_$rep.err; exit 1; }
    python -c "import json; r=json.load(open('$OUT/roof_${lib}_$rep.json'))['roofline']; print('$lib', r['frac'], r['ms_fwd'], r['ms_bwd'])"
  done
done
