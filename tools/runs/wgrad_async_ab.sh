# Side-stream weight gradients (TAGAN_WGRAD_ASYNC=1): parity (model-level GPU tests + graph replays), then
# interleaved C2 bench lines with and without
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-wgasync}
mkdir -p $OUT
TAGAN_WGRAD_ASYNC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_sharded.py tests/test_gpu_ingest.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for a in 1 0; do
    TAGAN_WGRAD_ASYNC=$a timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/b.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b.json')); print('async=$a', d['ms_per_step'], d['launch'], d['alt_precision']['ms_per_step'])"
  done
done
