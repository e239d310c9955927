#!/bin/bash
# Round 6 (w): the temporal bias table on csrc/params.hip.  Bias-table + temporal + parity tests, the default bench
# ABAB against the previous tree's library... (the gather GEMMs are the CPU path; A/B here = bench before / after
# from r6v4 on another box, so only the kernel stats are compared), per-kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bias_table.py tests/test_gpu_narrow.py tests/test_gpu_temporal_T.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 --no-roofline > $OUT/bench.$r.json 2> $OUT/bench.$r.err || { tail -20 $OUT/bench.$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench.$r.json'));print('run $r c2', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_trace*" -delete
python -c "
import csv
for r in csv.DictReader(open('$OUT/stats/run_kernel_stats.csv')):
    if 'bias_table' in r['Name'] or 'Cijk' in r['Name'] or 'elementwise' in r['Name']: print('  %-70s %5s %9.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))"
python tools/kstats.py $OUT/stats/run_kernel_stats.csv | sed -n 1,3p
