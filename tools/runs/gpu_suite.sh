#!/bin/bash
# the whole GPU test suite, one pytest process, into gpurun_out/<dir>/suite.log
set -o pipefail
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/suite.log | tail -5
tail -3 $OUT/suite.log
exit $rc
