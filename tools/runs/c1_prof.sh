# C1 step under rocprofv3 kernel stats (graph launch): where the 0.8 ms go
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/c1prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o run -- python bench.py --config c1 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-alt-precision --launch graph > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep -h '"metric"' $OUT/bench.log | cut -c1-200
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/c1prof/p/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last 30 steps: find k_head_fwd occurrences as step markers
idx = [i for i, r in enumerate(rows) if 'k_head_fwd' in r['Kernel_Name']]
a, b = idx[-11], idx[-1]
seg = rows[a:b]
n = 10
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg) / n / 1e3
span = (int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / n / 1e3
print('kernels/step %.1f  busy us/step %.1f  wall us/step %.1f' % (len(seg) / n, busy, span))
from collections import defaultdict
agg = defaultdict(lambda: [0, 0])
for r in seg:
    k = r['Kernel_Name'][:90]
    agg[k][0] += 1; agg[k][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print('%7.1f us %5.1f  %s' % (t / n / 1e3, c / n, k))
gaps = [int(seg[i+1]['Start_Timestamp']) - int(seg[i]['End_Timestamp']) for i in range(len(seg)-1)]
gaps.sort()
print('median gap us %.2f, p90 %.2f' % (gaps[len(gaps)//2]/1e3, gaps[int(len(gaps)*0.9)]/1e3))
PY
find $OUT/p -name "*kernel_trace*" -delete
