#!/bin/bash
# Round 5 (b): LDS-DMA staging of the K = 128 fp32-operand stream GEMMs (k_sgemm_ntg, libtagan_hip.so) against the
# round-4 register staging (libtagan_hip_noglds.so): stream-GEMM parity tests on the new default, the per-product
# probe on both, the C2 step interleaved (separate processes, same box), rocprof kernel stats of the new step; LAST,
# the forced watchdog race without the fix (tests/test_gpu_rccl.py capture_race_unfixed; expected: the abort).
#   bash tools/runs/r5b.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5b}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py tests/test_gpu_graph.py \
    -m gpu -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libtagan_hip.so libtagan_hip_noglds.so; do
  TAGAN_LIB=$L/$lib SGEMM_PROBE_OUT=$OUT/probe_$lib.json timeout -k 10 300 python tools/sgemm_probe.py \
      > $OUT/probe_$lib.log 2>&1 || { tail -20 $OUT/probe_$lib.log; exit 1; }
  echo "== probe $lib"; python -c "
import json;d=json.load(open('$OUT/probe_$lib.json'))
for c in d['cases']: print('%-16s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_noglds.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
find $OUT/stats -name "*kernel_trace*" -delete
f=$(find $OUT/stats -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f | sed -n 1,14p
python tools/sgemm_table.py $f > $OUT/sgemm_table_fp32.md; cat $OUT/sgemm_table_fp32.md
timeout -k 10 120 python -u tests/test_gpu_rccl.py capture_race_unfixed > $OUT/race_unfixed.log 2>&1; echo "unfixed race rc=$?"
grep -m3 -E "hipErrorCapturedEvent|capturing stream|RCCL_CASE_OK" $OUT/race_unfixed.log
exit 0
