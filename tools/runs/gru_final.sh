set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gru
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gru.py tests/test_gpu_tprop.py tests/test_gpu_sharded.py > gpurun_out/gru/final.log 2>&1 || { tail -30 gpurun_out/gru/final.log; exit 1; }
tail -1 gpurun_out/gru/final.log
for cfg in c2 c4; do for bi in 0 1; do
  timeout -k 10 300 python tools/tprop_probe.py --config $cfg --bidirectional $bi --reps 5 || exit 1
done; done | tee gpurun_out/gru/final_probe.jsonl
