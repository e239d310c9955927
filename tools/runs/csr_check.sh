#!/bin/bash
# CSR builder: bit-exact GPU tests, timing on C2/C4 batches, rocprofv3 kernel trace of the same.
# usage (on the GPU box, repo root): bash tools/runs/csr_check.sh <outdir under gpurun_out>
set -o pipefail
OUT=gpurun_out/${1:-csr}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k csr -x -v --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python -u tools/csr_bench.py --configs c2,c4 --out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep build_ms $OUT/bench.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run -- python3 $R/tools/csr_bench.py --configs c4,c2 --reps 3 > $R/$OUT/prof.log 2>&1
echo prof rc=$?
