#!/bin/bash
# one GPU test (node id in $2) with HIP runtime error logging, into gpurun_out/<dir>
set -o pipefail
OUT=gpurun_out/${1:-one}
mkdir -p $OUT
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest $2 -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?
grep -v "^$" $OUT/t.log | grep -iv "extension modules" | tail -40
exit $rc
