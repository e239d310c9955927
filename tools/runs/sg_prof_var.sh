#!/bin/bash
# rocprofv3 kernel stats (fp32 and bf16 C2 steps) per env variant: GEMM table + LayerNorm kernels.
# bash tools/runs/sg_prof_var.sh <tag> <variant>...   (variant = ENV=VAL[,ENV=VAL] or base)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sgpv}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  envs=""
  [ "$v" != "base" ] && envs=$(echo "$v" | tr ',' ' ')
  tag=$(echo "$v" | tr ',=' '_-')
  for prec in fp32 bf16; do
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_$prec -o run -- \
      python bench.py --steps 20 --warmup 3 --precision $prec --no-cpu-baseline --no-roofline --no-alt-precision \
      --no-c1 > $OUT/${tag}_$prec.log 2>&1 || { tail -20 $OUT/${tag}_$prec.log; exit 1; }
    find $OUT/${tag}_$prec -name "*kernel_trace*" -delete
    f=$(find $OUT/${tag}_$prec -name "*kernel_stats.csv" | head -1)
    echo "== $v $prec"
    python tools/kstats.py $f | sed -n 1,4p
    python tools/sgemm_table.py $f | tail -n +3
    python - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "k_ln_" in r["Name"] or "rowgemm" in r["Name"]:
        print("   %7.1f us x %5d  %s" % (float(r["TotalDurationNs"]) / int(r["Calls"]) / 1e3, int(r["Calls"]), r["Name"][:90]))
PY
  done
done
