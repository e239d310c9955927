#!/bin/bash
# default bench line + rocprof kernel stats of the C2 steps (one gpurun call) into gpurun_out/<dir>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-bs}
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/runs/c2_stats.sh ${1:-bs}
