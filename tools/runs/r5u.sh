#!/bin/bash
# Round 5 (u): block order of the edge chunk kernels (TAGAN_GEO_XCD): 1 = XCD-contiguous eighths of the capacity-sized
# grid (the shipped map: the valid chunks fill 75 % of it on the uniform graphs, so two XCDs idle), 2 = the same over
# the valid blocks only, 0 = launch order; edge-kernel tests, then the kernels alone at C2 / C4 / C3 / C5 (bf16),
# interleaved x2.   bash tools/runs/r5u.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5u}
mkdir -p $OUT
for m in 2 0; do
  TAGAN_GEO_XCD=$m timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 \
      --timeout-method thread -k "geo or gat or csr or edge" > $OUT/tests_$m.log 2>&1 || { tail -40 $OUT/tests_$m.log; exit 1; }
  echo "mode $m: $(tail -1 $OUT/tests_$m.log)"
done
for rep in 1 2; do
  for cfg in "c2" "c4" "c3" "c5 --bf16"; do
    for m in 1 2 0; do
      TAGAN_GEO_XCD=$m timeout -k 10 300 python tools/geo_kernels.py --config $cfg --reps 5 > $OUT/gk.log 2>&1 || { tail -20 $OUT/gk.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/gk.log').read().strip().splitlines()[-1]);print('$cfg xcd=$m', d['ms_fwd'], d['ms_bwd'], d.get('frac_hbm', d.get('frac')))"
    done
  done
done
