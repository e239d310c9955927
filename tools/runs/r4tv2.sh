#!/bin/bash
# TAGAN_V4_PREFETCH=1 (libtagan_hip_pf.so): the temporal / parity / graph / full-size GPU tests on it, then two
# interleaved C2 bench rounds against the shipped library.
#   bash tools/runs/r4tv2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4tv2}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_pf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_temporal_v4.py \
    tests/test_gpu_temporal_v5.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -m gpu \
    -x -q --timeout 200 --timeout-method thread > $OUT/tests_pf.log 2>&1 || { tail -40 $OUT/tests_pf.log; exit 1; }
tail -1 $OUT/tests_pf.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_pf.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
