#!/bin/bash
# Round-2 GPU call: GPU suite (optional), default bench line, rocprofv3 kernel stats of a short C2 bench.
# Outputs under gpurun_out/$1/.  SKIP_TESTS=1 skips pytest; BENCH_ARGS adds bench flags.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r2step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 20 \
      --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
  rc=$?
  tail -5 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c2 -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/stats_c2.log 2>&1 || { tail -20 $OUT/stats_c2.log; exit 1; }
find $OUT/stats_c2 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c2 -name "*kernel_stats.csv" | head -1) 7
du -sh $OUT
