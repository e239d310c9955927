set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tprop_prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in c2 c4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$cfg -o run -- python tools/tprop_probe.py --config $cfg --reps 5 --only gru_kernel > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
find $OUT/$cfg -name "*kernel_trace*" -delete
CFG=$cfg python - <<'PY'
import csv, glob, os
f = glob.glob('gpurun_out/tprop_prof/%s/**/*kernel_stats.csv' % os.environ['CFG'], recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
print(os.environ['CFG'], 'total ms per rep', round(sum(float(r['TotalDurationNs']) for r in rows) / 7e6, 3))
for r in rows[:14]:
    print('%9.3f ms/rep %6.1f calls/rep  %s' % (float(r['TotalDurationNs']) / 7e6, int(r['Calls']) / 7, r['Name'][:90]))
PY
done
