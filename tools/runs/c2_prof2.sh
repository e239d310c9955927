#!/bin/bash
# C2 bench line (no CPU baseline / roofline) + rocprofv3 kernel stats of the fp32 and bf16 steps + the stream-GEMM
# per-shape tables.  bash tools/runs/c2_prof2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c2p}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 > $OUT/bench.json \
    2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], d['alt_precision']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for prec in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s_$prec -o run -- \
    python bench.py --steps 20 --warmup 3 --precision $prec --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    > $OUT/s_$prec.log 2>&1 || { tail -20 $OUT/s_$prec.log; exit 1; }
  find $OUT/s_$prec -name "*kernel_trace*" -delete
  echo "== $prec"
  python tools/kstats.py $(find $OUT/s_$prec -name "*kernel_stats.csv" | head -1) | sed -n 1,14p
  python tools/sgemm_table.py $(find $OUT/s_$prec -name "*kernel_stats.csv" | head -1)
done
