#!/bin/bash
# CSR/CSC build on a side stream under the node embedding and the first block's QKV projection (TAGAN_CSR_SIDE=1,
# default) against in line (TAGAN_CSR_SIDE=0): the full GPU suite on the default, C2 fp32 / bf16 steps interleaved,
# C4 one line each.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zm}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -40 $OUT/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -n 1 $OUT/gpu_tests.log)"
for r in 1 2; do
  for S in 1 0; do
    for P in fp32 bf16; do
      TAGAN_CSR_SIDE=$S timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
          --no-roofline --no-alt-precision --no-c1 --precision $P > $OUT/b${S}_${P}_$r.json 2> $OUT/b${S}_${P}_$r.err \
          || { tail -20 $OUT/b${S}_${P}_$r.err; exit 1; }
      echo "side=$S $P run $r: $(python -c "import json;d=json.load(open('$OUT/b${S}_${P}_$r.json'));print(d['ms_per_step'], d.get('breakdown',{}).get('forward_ms'))")"
    done
  done
done
for S in 1 0; do
  TAGAN_CSR_SIDE=$S timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline \
      --no-alt-precision --no-c1 --launch eager > $OUT/c4_$S.json 2> $OUT/c4_$S.err || { tail -20 $OUT/c4_$S.err; exit 1; }
  echo "c4 side=$S: $(python -c "import json;d=json.load(open('$OUT/c4_$S.json'));print(d['ms_per_step'], d.get('breakdown'))")"
done
