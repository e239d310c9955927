set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gru
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gru.py > gpurun_out/gru/tests.log 2>&1 || { tail -30 gpurun_out/gru/tests.log; exit 1; }
TAGAN_GRU_MR=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gru.py > gpurun_out/gru/tests16.log 2>&1 || { tail -30 gpurun_out/gru/tests16.log; exit 1; }
tail -1 gpurun_out/gru/tests.log gpurun_out/gru/tests16.log
for mr in 32 16; do for cfg in c2 c4; do
  TAGAN_GRU_MR=$mr timeout -k 10 300 python tools/tprop_probe.py --config $cfg --reps 5 --only gru_kernel | sed "s/^/mr=$mr /" || exit 1
done; done
TAGAN_GRU_MFMA=0 timeout -k 10 300 python tools/tprop_probe.py --config c2 --reps 5 --only gru_kernel | sed "s/^/valu /"
