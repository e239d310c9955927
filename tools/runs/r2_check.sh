#!/bin/bash
# Round-2 GPU call: full GPU suite (observed parity errors -> parity_errors.json), the default bench line,
# rocprofv3 kernel stats of the C4 roofline launches and of the C2 bench, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the C4 roofline launches -> pmc_c4.json.  Outputs under gpurun_out/$1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r2chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != "1" ]; then
  TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 20 \
      --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
  rc=$?
  tail -5 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c4 -o run -- \
    python bench.py --roofline-only --roofline-reps 10 > $OUT/stats_c4.log 2>&1 || { tail -20 $OUT/stats_c4.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_c4 -- \
    python bench.py --roofline-only --roofline-reps 2 > $OUT/fetch_c4.log 2>&1 || { tail -20 $OUT/fetch_c4.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_c4 -- \
    python bench.py --roofline-only --roofline-reps 2 > $OUT/write_c4.log 2>&1 || { tail -20 $OUT/write_c4.log; exit 1; }
find $OUT/stats_c4 $OUT/fetch_c4 $OUT/write_c4 -name "*kernel_trace*" -delete
python tools/pmc_summary.py $OUT/fetch_c4 $OUT/write_c4 c4 $OUT/pmc_c4.json > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c2 -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/stats_c2.log 2>&1 || { tail -20 $OUT/stats_c2.log; exit 1; }
find $OUT/stats_c2 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c2 -name "*kernel_stats.csv" | head -1) 7
python tools/kstats.py $(find $OUT/stats_c4 -name "*kernel_stats.csv" | head -1) 1
du -sh $OUT
