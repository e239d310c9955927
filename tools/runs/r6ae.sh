#!/bin/bash
# Round 6 (ae): narrow tests; narrow backward workgroups (TAGAN_NARROW_BWD_GROUPS = 256 / 512 / 1024), C2 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6ae}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_narrow.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for g in 256 512 1024; do
  TAGAN_NARROW_BWD_GROUPS=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$g -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats_$g.log 2>&1 || { tail -20 $OUT/stats_$g.log; exit 1; }
  find $OUT/stats_$g -name "*kernel_trace*" -delete
  echo "groups $g: $(python -c "
import csv
for r in csv.DictReader(open('$OUT/stats_$g/run_kernel_stats.csv')):
    if 'k_narrow' in r['Name'] or 'colsum' in r['Name']: print('%s %.1f' % (r['Name'][35:52], float(r['AverageNs'])/1e3), end='  ')")"
done
