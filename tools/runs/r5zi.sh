#!/bin/bash
# Edge-kernel HBM traffic re-collected on the round-5 tree (the block order changed this round): the C4 roofline
# line + kernel stats + FETCH_SIZE / WRITE_SIZE passes (tools/runs/roof_pmc.sh -> pmc_c4.json), and the same two
# passes over the C2 graph (tools/roofline_kernels.py -> pmc_c2.json, the bench's cache_assisted traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5zi}
bash tools/runs/roof_pmc.sh ${1:-r5zi} || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_c2 -- \
    python tools/roofline_kernels.py c2 > $OUT/fetch_c2.log 2>&1 || { tail -20 $OUT/fetch_c2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_c2 -- \
    python tools/roofline_kernels.py c2 > $OUT/write_c2.log 2>&1 || { tail -20 $OUT/write_c2.log; exit 1; }
find $OUT/fetch_c2 $OUT/write_c2 -name "*kernel_trace*" -delete
python tools/pmc_summary.py $OUT/fetch_c2 $OUT/write_c2 c2 $OUT/pmc_c2.json > /dev/null
cat $OUT/pmc_c2.json
tail -n 2 $OUT/fetch_c2.log
