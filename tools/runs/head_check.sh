set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/head
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_head.py tests/test_gpu_window.py tests/test_gpu_graph.py > gpurun_out/head/tests.log 2>&1 || { tail -30 gpurun_out/head/tests.log; exit 1; }
tail -3 gpurun_out/head/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/head/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --launch graph > gpurun_out/head/bench.log 2>&1 || { tail -20 gpurun_out/head/bench.log; exit 1; }
tail -1 gpurun_out/head/bench.log | cut -c1-300
find gpurun_out/head/prof -name "*kernel_trace*" -delete
grep -h "k_head\|k_tattn" $(find gpurun_out/head/prof -name "*kernel_stats.csv") | cut -c1-200
