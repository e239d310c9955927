#!/bin/bash
# Round 6 (h): cold-batch forward features per lane.  Geo parity (warm + forced cold), block-order and full-size
# tests; edge kernels alone at C2 / C4 fp32 and C5 bf16 (its cold forward at 4 vs 8 features per lane via
# TAGAN_GEO_FPL_FWD_COLD); the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 \
    --timeout-method thread -k "geo or fullsize_model or sampled" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for c in c2 c4; do
    timeout -k 10 300 python tools/geo_kernels.py --config $c --reps 10 > $OUT/geo_$c.$r.json 2>&1 || { tail -5 $OUT/geo_$c.$r.json; exit 1; }
    echo "$c fp32 run $r: $(tail -1 $OUT/geo_$c.$r.json)"
  done
  for f in 8 4; do
    TAGAN_GEO_FPL_FWD_COLD=$f timeout -k 10 300 python tools/geo_kernels.py --config c5 --bf16 --reps 5 > $OUT/geo_c5_f$f.$r.json 2>&1 || { tail -5 $OUT/geo_c5_f$f.$r.json; exit 1; }
    echo "c5 bf16 cold fwd FPL $f run $r: $(tail -1 $OUT/geo_c5_f$f.$r.json)"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));R=d['roofline'];print('bench c2', d['ms_per_step'], d['alt_precision']['ms_per_step'], 'c4 roofline fwd/bwd', R['ms_fwd'], R['ms_bwd'], R['frac'])"
