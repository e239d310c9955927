#!/bin/bash
# Head kernel phase stamps (instrumented libtagan_hip_hprof.so) at the C2 head and a larger one.
#   bash tools/runs/r4hp.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4hp}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_hprof.so timeout -k 10 200 python tools/head_probe.py --reps 4 > $OUT/c2.txt 2>&1 \
    || { tail -20 $OUT/c2.txt; exit 1; }
tail -4 $OUT/c2.txt
TAGAN_LIB=$L/libtagan_hip_hprof.so timeout -k 10 200 python tools/head_probe.py --reps 3 --H 256 > $OUT/h256.txt 2>&1 \
    || { tail -20 $OUT/h256.txt; exit 1; }
tail -2 $OUT/h256.txt
