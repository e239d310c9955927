#!/bin/bash
# Round 6 (q): merge kernels (k_geo_fwd_merge / k_geo_sum_parts) with branch-free chunk loads and G = 4 / 8 / 16
# accumulators per lane (TAGAN_GEO_MG).  Geo parity + block-order tests, the edge passes alone at C2 / C4 per G,
# per-kernel stats of the C2 edge passes per G, the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 \
    --timeout-method thread -k "geo or fullsize_model or sampled" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for g in 4 8 16; do
    for c in c2 c4; do
      TAGAN_GEO_MG=$g timeout -k 10 300 python tools/geo_kernels.py --config $c --reps 10 > $OUT/geo_${c}_g$g.$r.json 2>&1 || { tail -5 $OUT/geo_${c}_g$g.$r.json; exit 1; }
      echo "$c G=$g run $r: $(tail -1 $OUT/geo_${c}_g$g.$r.json)"
    done
  done
done
for g in 4 8 16; do
  TAGAN_GEO_MG=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_g$g -o k -- python tools/geo_kernels.py --config c2 --reps 10 > $OUT/prof_g$g.log 2>&1 || { tail -5 $OUT/prof_g$g.log; exit 1; }
  f=$(find $OUT/prof_g$g -name '*kernel_stats.csv' | head -1)
  cp $f $OUT/c2_geo_kstats_g$g.csv
  echo "G=$g: $(grep -E 'k_geo_sum_parts|k_geo_fwd_merge' $f | cut -d, -f1-5 | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));R=d['roofline'];print('bench c2', d['ms_per_step'], d['alt_precision']['ms_per_step'], 'c4 roofline fwd/bwd', R['ms_fwd'], R['ms_bwd'], R['frac'])"
