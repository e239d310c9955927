#!/bin/bash
# stream-GEMM iteration: unit tests, same-process LN-variant A/B (fp32 + bf16), kernel stats of the default step.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sgi}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 120 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
for prec in fp32 bf16; do
  timeout -k 10 300 python tools/ab_step.py --precision $prec none in+out all > $OUT/ab_$prec.log 2>&1 \
      || { tail -20 $OUT/ab_$prec.log; exit 1; }
  grep median $OUT/ab_$prec.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for prec in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s_$prec -o run -- \
    python bench.py --steps 20 --warmup 3 --precision $prec --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/s_$prec.log 2>&1 || { tail -20 $OUT/s_$prec.log; exit 1; }
  find $OUT/s_$prec -name "*kernel_trace*" -delete
  f=$(find $OUT/s_$prec -name "*kernel_stats.csv" | head -1)
  echo "== $prec"; python tools/kstats.py $f | sed -n 1,6p
  python - $f <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"k_(sgemm_nt|sgemm_tn|rowgemm|ln_bwd|ln_fwd)<[^>]*>", r["Name"])
    if m:
        print("   %7.1f us x %4d  %s" % (float(r["TotalDurationNs"]) / int(r["Calls"]) / 1e3, int(r["Calls"]), m.group(0)))
PY
done
