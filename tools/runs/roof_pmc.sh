#!/bin/bash
# C4 edge-kernel roofline line (HIP events) + its rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes ->
# pmc_c4.json (tools/pmc_summary.py).  bash tools/runs/roof_pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-roof}
mkdir -p $OUT
timeout -k 10 200 python bench.py --roofline-only --roofline-reps 10 > $OUT/roof.json 2> $OUT/roof.err \
    || { tail -20 $OUT/roof.err; exit 1; }
python -c "import json; r=json.load(open('$OUT/roof.json'))['roofline']; print('frac', r['frac'], 'ms', r['ms_fwd'], r['ms_bwd'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c4 -o run -- \
    python bench.py --roofline-only --roofline-reps 10 > $OUT/stats_c4.log 2>&1 || { tail -20 $OUT/stats_c4.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_c4 -- \
    python bench.py --roofline-only --roofline-reps 2 > $OUT/fetch_c4.log 2>&1 || { tail -20 $OUT/fetch_c4.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_c4 -- \
    python bench.py --roofline-only --roofline-reps 2 > $OUT/write_c4.log 2>&1 || { tail -20 $OUT/write_c4.log; exit 1; }
find $OUT/stats_c4 $OUT/fetch_c4 $OUT/write_c4 -name "*kernel_trace*" -delete
python tools/pmc_summary.py $OUT/fetch_c4 $OUT/write_c4 c4 $OUT/pmc_c4.json > /dev/null
cat $OUT/pmc_c4.json
python tools/kstats.py $(find $OUT/stats_c4 -name "*kernel_stats.csv" | head -1) 1
