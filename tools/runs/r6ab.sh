#!/bin/bash
# Round 6 (ab): the fused head with 512-thread workgroups (TAGAN_HEAD_HB=512: no register spills in the backward,
# 128 VGPRs at 1024 threads spilled 64-188 B) against the shipped 1024: head tests on the variant, per-kernel
# stats of the C2 step per library, the default bench ABAB.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6ab}
mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_hb512.so
TAGAN_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in old new; do
  if [ $v = new ]; then L=$V; else L=; fi
  TAGAN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats_$v.log 2>&1 || { tail -20 $OUT/stats_$v.log; exit 1; }
  find $OUT/stats_$v -name "*kernel_trace*" -delete
  echo "$v:"; python -c "
import csv
for r in csv.DictReader(open('$OUT/stats_$v/run_kernel_stats.csv')):
    if 'k_head' in r['Name']: print('  %-50s %5s %9.1f' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
done
for r in 1 2; do
  for v in old new; do
    if [ $v = new ]; then L=$V; else L=; fi
    TAGAN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 --no-roofline > $OUT/bench_$v.$r.json 2> $OUT/bench_$v.$r.err || { tail -20 $OUT/bench_$v.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_$v.$r.json'));print('$v run $r c2', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
