#!/bin/bash
# Round 6 (y): the narrow embedding at H = 256 (two 128-column passes): C3 fp32 and C5 bf16 steps, ABAB against
# TAGAN_NARROW=0 (hipBLASLt forward + split-K weight gradient + bias column sum).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6y}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_narrow.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in 0 1; do
    for cp in "c3 fp32" "c5 bf16"; do
      set -- $cp
      TAGAN_NARROW=$v timeout -k 10 400 python bench.py --config $1 --precision $2 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager > $OUT/$1_$v.$r.json 2> $OUT/$1_$v.$r.err || { tail -20 $OUT/$1_$v.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/$1_$v.$r.json'));print('$1 $2 narrow=$v run $r', d['ms_per_step'])"
    done
  done
done
