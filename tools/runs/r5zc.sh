#!/bin/bash
# Round 5 (zc): rehearsal of the current tree (tools/runs/round_end.sh) followed by the C3 / C4 / C5 bench lines
# (tools/runs/c3c4c5_bench.sh).   bash tools/runs/r5zc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/runs/round_end.sh ${1:-r5zc} || exit 1
bash tools/runs/c3c4c5_bench.sh ${1:-r5zc}_c345 || exit 1
