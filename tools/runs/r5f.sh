#!/bin/bash
# Round 5 (f): the fp32 QKV input gradient with LN1's backward in its epilogue (weight-stationary k_sgemm_nt
# MODE_LN_BWD, three planes; epilogue operands loaded after the MFMAs, unconditional dres load): LN-fusion tests, the
# backward parity suites, and the same-process step A/B with and without "bwd" in fp32.   bash tools/runs/r5f.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5f}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_sgemm_ln.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/ab_step.py --precision fp32 in+out+ln2bwd all > $OUT/ab_fp32.log 2>&1 || { tail -20 $OUT/ab_fp32.log; exit 1; }
grep -i median $OUT/ab_fp32.log
