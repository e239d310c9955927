#!/bin/bash
# Edge-kernel change check (one gpurun call): the GPU tests that run the geometric kernels, the C4 roofline line
# (HIP events) and its rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes.  Outputs under gpurun_out/$1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-geo}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py \
    tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python bench.py --roofline-only --roofline-reps 10 > $OUT/roof.json 2> $OUT/roof.err \
    || { tail -20 $OUT/roof.err; exit 1; }
cat $OUT/roof.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --no-c1 > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('C2', d['ms_per_step'], 'ms; bf16', d['alt_precision']['ms_per_step'], 'ms', d['breakdown'])"
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
