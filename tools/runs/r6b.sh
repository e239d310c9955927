#!/bin/bash
# Round 6 (b): the round-5 dgamma determinism probe on two reconstructions of k_ln2_bwd_out's first form
# (TAGAN_LN2_FORM=1: next tile's loads after the plane-writing barriers; =2: also dead rows branched around) and the
# shipped form.
set -o pipefail
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for lib in libtagan_hip_l2f1.so libtagan_hip_l2f2.so libtagan_hip.so; do
  echo "== $lib"
  TAGAN_LIB=$L/$lib timeout -k 10 120 python -u tools/ln2_debug_probe.py 2>&1 | grep "skip=True" || exit 1
done
