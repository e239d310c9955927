#!/bin/bash
# In-step A/B of three library builds (separate processes, interleaved, same box): the shipped library (DPP / permlane
# lane reductions, whole-row A loads, split-K accumulation as its own instantiation), libtagan_hip_rl0.so (the same
# with the round-3 A load map) and libtagan_hip_nodpp.so (the previous build: shuffle reductions, runtime accumulate
# branch); the GPU suite on the shipped library first; rocprofv3 kernel stats of the C2 step for the first two.
#   bash tools/runs/r4i.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4i}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
LIBS="libtagan_hip.so libtagan_hip_rl0.so libtagan_hip_nodpp.so"
for rep in 1 2; do
  for lib in $LIBS; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in libtagan_hip.so libtagan_hip_rl0.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$lib -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
      > $OUT/stats_$lib.log 2>&1 || { tail -20 $OUT/stats_$lib.log; exit 1; }
  find $OUT/stats_$lib -name "*kernel_trace*" -delete
  echo "== $lib"
  python tools/kstats.py $(find $OUT/stats_$lib -name "*kernel_stats.csv" | head -1) | sed -n 1,12p
  python tools/sgemm_table.py $(find $OUT/stats_$lib -name "*kernel_stats.csv" | head -1)
done
