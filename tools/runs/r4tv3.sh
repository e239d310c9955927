#!/bin/bash
# v6 temporal kernels (C2: v6 forward; C4: v6 forward and backward) in fp32 and bf16 storage: shipped library against
# TAGAN_V6_PREFETCH=1 (next unit's slab share in registers) and TAGAN_V6_WPE=3 (waves per SIMD), two interleaved
# rounds.
#   bash tools/runs/r4tv.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4tv3}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_v6pf.so libtagan_hip_v6w3.so; do
    for cfg in c2 c4; do for dt in "" "--bf16"; do
      TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 20 $dt \
          > $OUT/t_${lib}_${cfg}_${rep}${dt}.json 2>&1 || { tail -5 $OUT/t_${lib}_${cfg}_${rep}${dt}.json; exit 1; }
      echo "$lib $cfg $dt $(python -c "import json;d=json.loads(open('$OUT/t_${lib}_${cfg}_${rep}${dt}.json').read().strip().splitlines()[-1]);print(d['ms_fwd'], d['ms_bwd'], d['checksums'])")"
    done; done
  done
done
