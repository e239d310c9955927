#!/bin/bash
# Round 6 (r): A/B of the branch-free merge kernels against the r6p library (tools/probes/libtagan_r6p.so, built
# from the previous geo_attn.hip): edge passes at C2 / C4 (one snapshot and all 16), the default bench line ABAB,
# per-kernel stats of the C2 step on the new library.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6r}
mkdir -p $OUT
export TMPDIR=/tmp
OLD=$PWD/tools/probes/libtagan_r6p.so
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=; fi
    for c in "c2" "c4 --snapshots 1" "c4"; do
      n=$(echo $c | tr -d ' -')
      TAGAN_LIB=$L timeout -k 10 300 python tools/geo_kernels.py --config $c --reps 10 > $OUT/geo_${n}_$v.$r.json 2>&1 || { tail -5 $OUT/geo_${n}_$v.$r.json; exit 1; }
      echo "$v $c run $r: $(tail -1 $OUT/geo_${n}_$v.$r.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_fwd"],d["ms_bwd"],d["frac"])')"
    done
  done
done
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=; fi
    TAGAN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c1 > $OUT/bench_$v.$r.json 2> $OUT/bench_$v.$r.err || { tail -20 $OUT/bench_$v.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_$v.$r.json'));R=d['roofline'];print('$v bench c2', d['ms_per_step'], d['alt_precision']['ms_per_step'], 'c4 roofline fwd/bwd', R['ms_fwd'], R['ms_bwd'], R['frac'])"
  done
done
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=; fi
  TAGAN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 > $OUT/stats_$v.log 2>&1 || { tail -20 $OUT/stats_$v.log; exit 1; }
  find $OUT/stats_$v -name "*kernel_trace*" -delete; f=$OUT/stats_$v/run_kernel_stats.csv
  echo "$v: $(python tools/kstats.py $f | sed -n 1,3p | tr '\n' ' ')"
  grep -E 'k_geo_(sum_parts|fwd_merge|bwd_col|bwd_row|fwd_chunk)' $f | cut -d, -f1-4 | cut -c1-160
done
