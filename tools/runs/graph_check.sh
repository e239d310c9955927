#!/bin/bash
# graph-replay checks: the GPU graph tests and repeated replays of the captured C2 step (capture / destroy / re-capture)
# graph-step robustness: graph tests (warnings shown), the default bench, then a long-replay bench (auto trial)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/gcheck
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_rccl.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
grep -c "AccumulateGrad" $OUT/tests.log || true
timeout -k 10 400 python bench.py --no-cpu-baseline --no-roofline > $OUT/b.json 2> $OUT/b.err || { grep -v "^frame" $OUT/b.err | tail -20; exit 1; }
grep -c "AccumulateGrad" $OUT/b.err || true
python -c "import json; d=json.load(open('$OUT/b.json')); print('default', d['ms_per_step'], d['launch'], d.get('launch_trial'), d['alt_precision']['ms_per_step'])"
timeout -k 10 400 python bench.py --steps 80 --warmup 5 --no-cpu-baseline --no-roofline --no-alt-precision > $OUT/b80.json 2> $OUT/b80.err || { grep -v "^frame" $OUT/b80.err | tail -20; exit 1; }
python -c "import json; d=json.load(open('$OUT/b80.json')); print('steps80', d['ms_per_step'], d['launch'])"
