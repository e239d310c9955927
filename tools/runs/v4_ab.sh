set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v4b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_T.py > gpurun_out/v4b/tests.log 2>&1 || { tail -30 gpurun_out/v4b/tests.log; exit 1; }
tail -3 gpurun_out/v4b/tests.log
for cfg in c2 c4 c1; do
  for v in 1 0; do
    TAGAN_TATTN_V4=$v timeout -k 10 120 python tools/tattn_kernels.py --config $cfg --reps 20 > gpurun_out/v4b/k_${cfg}_v$v.json 2>/dev/null || exit 1
    echo "$cfg v4=$v $(cat gpurun_out/v4b/k_${cfg}_v$v.json)"
  done
done
