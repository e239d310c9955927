#!/bin/bash
# Round 5 (a): the capture-time watchdog abort.  1) the HIP event-query semantics probe (no process group);
# 2) the RCCL test file, including the forced race with the fix; 3) the whole GPU suite and the bounds-check parity
# subset on HEAD, without -x; 4) LAST: the forced race WITHOUT the fix (expected: the watchdog abort, rc -6).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5a}
mkdir -p $OUT
timeout -k 10 120 python -u tools/captured_event_probe.py --out $OUT/captured_event_probe.json > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
cat $OUT/captured_event_probe.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 300 --timeout-method thread > $OUT/rccl.log 2>&1 || { tail -60 $OUT/rccl.log; exit 1; }
grep -E "PASS|FAIL" $OUT/rccl.log
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 1
TAGAN_LIB=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_debug.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membank.py tests/test_gpu_ingest.py \
    tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py tests/test_gpu_sgemm.py tests/test_gpu_debug.py \
    tests/test_gpu_head.py -m gpu \
    -q --timeout 300 --timeout-method thread > $OUT/debug_tests.log 2>&1 || { tail -40 $OUT/debug_tests.log; exit 1; }
tail -1 $OUT/debug_tests.log
timeout -k 10 120 python -u tests/test_gpu_rccl.py capture_race_unfixed > $OUT/race_unfixed.log 2>&1; echo "unfixed race rc=$?"
grep -m3 -E "hipErrorCapturedEvent|watchdog|RCCL_CASE_OK" $OUT/race_unfixed.log
exit 0
