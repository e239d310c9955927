#!/bin/bash
# Round 5 (v): the edge kernels' block order chosen by working set (launch order when the batch's K | V exceed the
# Infinity Cache, XCD-contiguous over the valid blocks otherwise): GPU parity / full-size / graph tests, the default
# bench line (C2 + the C4 roofline record), then C3 / C4 / C5 (bf16) steps with the chosen order and with the shipped
# map forced (TAGAN_GEO_XCD=1).   bash tools/runs/r5v.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5v}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py -m gpu -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('c2', d['value'], d['ms_per_step'], d['alt_precision']['ms_per_step'], 'roofline', d['roofline']['frac'])"
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for x in "" 1; do
  for c in "c3" "c4" "c5 --precision bf16"; do
    n=$(echo $c | cut -d' ' -f1)
    TAGAN_GEO_XCD=$x timeout -k 10 500 python bench.py --config $c $B > $OUT/${n}_x$x.json 2> $OUT/${n}_x$x.err || { tail -20 $OUT/${n}_x$x.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${n}_x$x.json'));print('$n xcd=${x:-auto}', d['ms_per_step'], d['value'])"
  done
done
