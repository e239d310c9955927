# Which GEMM kernels run in eager vs graph-captured steps (TunableOp table lookups inside capture?)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ggc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mode in eager graph; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$mode -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --launch $mode > $OUT/$mode.log 2>&1 || { tail $OUT/$mode.log; exit 1; }
  find $OUT/$mode -name "*kernel_trace*" -delete
  echo "== $mode $(grep -h '"metric"' $OUT/$mode.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  MODE=$mode python - <<'PY'
import csv, glob, os
f = glob.glob('gpurun_out/ggc/%s/**/*kernel_stats.csv' % os.environ['MODE'], recursive=True)[0]
rows = list(csv.DictReader(open(f)))
steps = [int(r['Calls']) for r in rows if 'k_head_fwd' in r['Name']][0]
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    if 'Cijk' in r['Name']:
        print('%6.3f ms/step %5.2f calls %7.1f us  %s' % (float(r['TotalDurationNs']) / 1e6 / steps, int(r['Calls']) / steps,
                                                       float(r['AverageNs']) / 1e3, r['Name'][:80]))
PY
done
