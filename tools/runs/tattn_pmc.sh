#!/bin/bash
# temporal kernel timing + SQ counter passes at one config: bash tools/runs/tattn_pmc.sh <tag> <config>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sq_$1
timeout -k 10 300 python tools/tattn_kernels.py --config $2 --reps 5 > gpurun_out/sq_$1/time.json 2>&1 || { tail -5 gpurun_out/sq_$1/time.json; exit 1; }
cat gpurun_out/sq_$1/time.json
bash tools/sq_counters.sh $1 python tools/tattn_kernels.py --config $2 --reps 1
cat gpurun_out/sq_$1/table.txt
