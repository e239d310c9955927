#!/bin/bash
# C2 temporal kernels (v6 forward, v4 backward) in fp32 and bf16 storage: shipped library against compile-time v4
# backward variants (TAGAN_V4_PREFETCH=1: next row's operands in flight; TAGAN_V4_WPE_B=2 / 4 waves per EU), two
# interleaved rounds.
#   bash tools/runs/r4tv.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4tv}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_pf.so libtagan_hip_wpe2.so libtagan_hip_wpe4.so; do
    for dt in "" "--bf16"; do
      TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/tattn_kernels.py --config c2 --reps 20 $dt \
          > $OUT/t_${lib}_${rep}${dt}.json 2>&1 || { tail -5 $OUT/t_${lib}_${rep}${dt}.json; exit 1; }
      echo "$lib $dt $(python -c "import json;d=json.loads(open('$OUT/t_${lib}_${rep}${dt}.json').read().strip().splitlines()[-1]);print(d['ms_fwd'], d['ms_bwd'], d['checksums'])")"
    done
  done
done
