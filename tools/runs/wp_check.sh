#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-wpc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread \
    > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 > $OUT/b.json 2> $OUT/b.err \
    || { tail -20 $OUT/b.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['ms_per_step'], d['alt_precision']['ms_per_step'])"
