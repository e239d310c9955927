#!/bin/bash
# Round 5 (z): fp32 weight-stationary NT staging the next tile during the second half of the MFMAs (split VALU and LDS writes interleaved by scheduling groups)
# (libtagan_hip_ilv.so, TAGAN_SG_ILV=1) against the stash after the MFMAs: stream-GEMM tests on the
# variant, per-product probe on both, the C2 step interleaved (separate processes).   bash tools/runs/r5z.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5z}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_LIB=$L/libtagan_hip_ilv.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py \
    tests/test_gpu_sgemm_ln.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libtagan_hip.so libtagan_hip_ilv.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/sgemm_probe.py --planes 3,1 --cases qkv_fwd,qkv_fwd_ln,dh,out_fwd \
      > $OUT/probe_$lib.log 2>&1 || { tail -20 $OUT/probe_$lib.log; exit 1; }
  echo "== probe $lib"; python -c "
import json
for l in open('$OUT/probe_$lib.log'):
    if l.startswith('{'):
        c = json.loads(l); print('%-22s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_ilv.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
