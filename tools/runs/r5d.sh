#!/bin/bash
# Round 5 (d): dgamma determinism probe (tools/ln2_debug_probe.py) of three k_ln2_bwd_out builds -> profiles/r5d_ln2_probe.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for lib in libtagan_hip.so libtagan_hip_l2v1.so libtagan_hip_l2v2.so; do
  echo "== $lib"
  TAGAN_LIB=$L/$lib timeout -k 10 120 python -u tools/ln2_debug_probe.py 2>&1 | grep "skip=True" || exit 1
done
