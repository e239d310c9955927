#!/bin/bash
# One GPU call: rocprofv3 kernel stats of the C2 bench + the two PMC passes (FETCH_SIZE, WRITE_SIZE)
# of the edge kernels for roofline.traffic + the C4 roofline run.  Outputs under gpurun_out/prof_$1/.
set -e
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/stats.log 2>&1
find $OUT/stats -name "*kernel_trace*" -delete
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -- \
    python tools/geo_kernels.py --config c2 --reps 2 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -- \
    python tools/geo_kernels.py --config c2 --reps 2 > $OUT/write.log 2>&1
find $OUT/fetch $OUT/write -name "*kernel_trace*" -delete
python tools/pmc_summary.py $OUT/fetch $OUT/write c2 $OUT/pmc_c2.json > /dev/null
timeout -k 10 300 python tools/geo_kernels.py --config c4 > $OUT/geo_c4.json
timeout -k 10 300 python tools/tattn_kernels.py --config c2 > $OUT/tattn_c2.json
timeout -k 10 300 python tools/tattn_kernels.py --config c4 > $OUT/tattn_c4.json
du -sh $OUT
