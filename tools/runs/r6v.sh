#!/bin/bash
# Round 6 (v): the node embedding on csrc/narrow.hip (exact-f32 MFMA forward; dW | db in one pass).  Narrow parity
# tests, the model-level parity / full-size tests, the default bench ABAB against TAGAN_NARROW=0, per-kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6v}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in 0 1; do
    TAGAN_NARROW=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 --no-roofline > $OUT/bench_$v.$r.json 2> $OUT/bench_$v.$r.err || { tail -20 $OUT/bench_$v.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_$v.$r.json'));print('narrow=$v run $r c2', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_trace*" -delete
python -c "
import csv
for r in csv.DictReader(open('$OUT/stats/run_kernel_stats.csv')):
    if 'narrow' in r['Name'] or 'colsum' in r['Name']: print('  %-60s %5s %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
python tools/kstats.py $OUT/stats/run_kernel_stats.csv | sed -n 1,3p
