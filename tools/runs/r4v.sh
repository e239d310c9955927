#!/bin/bash
# CSR / CSC big-bucket finish with 1024-thread workgroups (libtagan_hip_bnt1k.so, 134 KB of dynamic LDS) against the
# shipped 512 threads / 140 KB: the CSR GPU tests on the variant, then csr_bench C2 / C4 and the C2 step, interleaved x2.
#   bash tools/runs/r4v.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4v}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_bnt1k.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "csr" \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_bnt1k.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/csr_bench.py --configs c2,c4 --reps 10 > $OUT/csr_${lib}_$rep.json 2>&1 \
        || { tail -5 $OUT/csr_${lib}_$rep.json; exit 1; }
    echo "$lib"; grep build_ms $OUT/csr_${lib}_$rep.json | cut -c1-160
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        --no-alt-precision > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['breakdown']['csr_build_ms'])"
  done
done
