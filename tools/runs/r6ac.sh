#!/bin/bash
# Round 6 (ac): narrow embedding forward grid (TAGAN_NARROW_GRID = 256 / 512 / 768 / 1024 workgroups), C2 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6ac}
mkdir -p $OUT
export TMPDIR=/tmp
for g in 256 512 768 1024; do
  TAGAN_NARROW_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$g -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats_$g.log 2>&1 || { tail -20 $OUT/stats_$g.log; exit 1; }
  find $OUT/stats_$g -name "*kernel_trace*" -delete
  echo "grid $g: $(python -c "
import csv
for r in csv.DictReader(open('$OUT/stats_$g/run_kernel_stats.csv')):
    if 'k_narrow' in r['Name']: print('%s %.1f' % (r['Name'][35:52], float(r['AverageNs'])/1e3), end='  ')")"
done
