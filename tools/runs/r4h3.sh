#!/bin/bash
# Head kernels: float4 staging copies (shipped library) against scalar batched copies (libtagan_hip_nu.so)
# and the previous commit (libtagan_hip_prevhead.so):
# head GPU tests, then per library a kernel-trace profile of the C2 bench and two
# interleaved bench runs.
#   bash tools/runs/r4h.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4h3}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/test_head.log 2>&1 || { tail -30 $OUT/test_head.log; exit 1; }
tail -2 $OUT/test_head.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in libtagan_hip.so libtagan_hip_prevhead.so libtagan_hip_nu.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o run \
      -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-c1 \
      > $OUT/prof_$lib.log 2>&1 || { tail -20 $OUT/prof_$lib.log; exit 1; }
  find $OUT/prof_$lib -name "*kernel_trace*" -delete
  python - $OUT/prof_$lib <<'EOF'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_head" in r["Name"]:
            print(sys.argv[1].split("prof_")[-1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
EOF
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_prevhead.so libtagan_hip_nu.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'])"
  done
done
