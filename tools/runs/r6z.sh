#!/bin/bash
# Round 6 (z): CSR row-slot counting wave-aggregated for the wave's first row (TAGAN_CSR_AGG) against =0;
# graph tests (bit-exact CSR/CSC), csr_bench ABAB against the =0 variant, per-kernel stats of
# the C2 CSR build per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6z}
mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_noagg.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py -m gpu -q -x --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$V; else L=; fi
    TAGAN_LIB=$L timeout -k 10 300 python tools/csr_bench.py --configs c2,c4 --reps 20 > $OUT/csr_$v.$r.json 2>&1 || { tail -5 $OUT/csr_$v.$r.json; exit 1; }
    echo "$v run $r: $(cat $OUT/csr_$v.$r.json | tr '\n' ' ' | cut -c1-600)"
  done
done
for v in old new; do
  if [ $v = old ]; then L=$V; else L=; fi
  TAGAN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o run -- \
      python tools/csr_bench.py --configs c2 --reps 20 > $OUT/stats_$v.log 2>&1 || { tail -20 $OUT/stats_$v.log; exit 1; }
  find $OUT/stats_$v -name "*kernel_trace*" -delete
  echo "$v:"; python -c "
import csv
for r in csv.DictReader(open('$OUT/stats_$v/run_kernel_stats.csv')):
    if 'k_c' in r['Name'] or 'k_part' in r['Name'] or 'k_big' in r['Name'] or 'k_refine' in r['Name']: print('  %-40s %5s %9.1f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
