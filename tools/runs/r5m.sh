#!/bin/bash
# Round 5 (m): where the fp32 weight-stationary NT time goes -- diagnostic builds (wrong results, timing only):
# diag1 one plane product instead of six, diag2 one plane read per fragment, diag3 no plane split in the stash,
# diag4 no output stores; against the shipped build.   bash tools/runs/r5m.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5m}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for lib in libtagan_hip.so libtagan_hip_diag1.so libtagan_hip_diag2.so libtagan_hip_diag3.so libtagan_hip_diag4.so libtagan_hip.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/sgemm_probe.py --planes 3 --cases qkv_fwd,dh,out_fwd \
      > $OUT/probe_$lib.log 2>&1 || { tail -20 $OUT/probe_$lib.log; exit 1; }
  echo "== probe $lib"; python -c "
import json
for l in open('$OUT/probe_$lib.log'):
    if l.startswith('{'):
        c = json.loads(l); print('%-22s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
done
