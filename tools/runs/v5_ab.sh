# v5 temporal kernels: parity tests, then kernel times v5 vs v3 at C3 / C5 and v5 (mode 2) vs v4 at C2 / C1.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v5ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_temporal_v5.py \
    tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_T.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for cfg in c3 c5; do
  for v in 1 0; do
    TAGAN_TATTN_V5=$v timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 10 > $OUT/k_${cfg}_v5$v.json 2>$OUT/k_${cfg}_v5$v.err || { tail $OUT/k_${cfg}_v5$v.err; exit 1; }
    echo "$cfg V5=$v $(cat $OUT/k_${cfg}_v5$v.json)"
  done
done
for cfg in c2; do
  for v in 2 1; do
    TAGAN_TATTN_V5=$v timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k_${cfg}_v5$v.json 2>$OUT/k_${cfg}_v5$v.err || { tail $OUT/k_${cfg}_v5$v.err; exit 1; }
    echo "$cfg V5=$v $(cat $OUT/k_${cfg}_v5$v.json)"
  done
done
