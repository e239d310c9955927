#!/bin/bash
# LN-fused stream GEMMs: unit tests, the model-level parity tests that run the fused blocks (every op fused), and an
# interleaved C2 A/B over TAGAN_SG_LN = 0 | in | in,out | all.  bash tools/runs/sgln_check.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sgln}
mkdir -p $OUT
if [ -z "$2" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm_ln.py -q --timeout 120 --timeout-method thread \
    > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -2 $OUT/unit.log
TAGAN_SG_LN=all timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_gpu_bf16.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 \
    || { tail -40 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
fi
for r in 1 2; do
  for v in 0 in in,out all; do
    TAGAN_SG_LN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -20 $OUT/b_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${v}_$r.json'));print('SG_LN=$v', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
