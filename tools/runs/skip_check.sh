#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-skc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_head.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q \
    --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for prec in fp32 bf16; do
  timeout -k 10 300 python tools/ab_step.py --precision $prec auto auto/skip0 > $OUT/ab_$prec.log 2>&1 \
      || { tail -20 $OUT/ab_$prec.log; exit 1; }
  grep median $OUT/ab_$prec.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s_fp32 -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/s_fp32.log 2>&1 || { tail -20 $OUT/s_fp32.log; exit 1; }
find $OUT/s_fp32 -name "*kernel_trace*" -delete
f=$(find $OUT/s_fp32 -name "*kernel_stats.csv" | head -1)
python tools/kstats.py $f | sed -n 1,3p
python - $f <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"k_(head_fwd|head_bwd|ln_bwd)[^(]*", r["Name"])
    if m:
        print("   %7.1f us x %4d  %s" % (float(r["TotalDurationNs"]) / int(r["Calls"]) / 1e3, int(r["Calls"]), m.group(0)))
PY
