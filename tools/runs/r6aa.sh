#!/bin/bash
# Round 6 (aa): edge kernels with 2 (shipped) / 3 / 4 edges unrolled per lane at 4 features per lane
# (TAGAN_GEO_UNROLL variant libraries): C4 one snapshot, C4 all 16, C2, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6aa}
mkdir -p $OUT
P=$PWD/temporal-asymmetric-graph-attention-network_amd
for r in 1 2; do
  for v in un2 un3 un4; do
    if [ $v = un2 ]; then L=; else L=$P/libtagan_hip_$v.so; fi
    for c in "c4 --snapshots 1" "c2"; do
      n=$(echo $c | tr -d ' -')
      TAGAN_LIB=$L timeout -k 10 300 python tools/geo_kernels.py --config $c --reps 10 > $OUT/geo_${n}_$v.$r.json 2>&1 || { tail -5 $OUT/geo_${n}_$v.$r.json; exit 1; }
      echo "$v $c run $r: $(tail -1 $OUT/geo_${n}_$v.$r.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_fwd"],d["ms_bwd"],d["frac"])')"
    done
  done
done
