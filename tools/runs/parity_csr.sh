#!/bin/bash
# GPU parity suite (test_gpu_parity.py) + the CSR builder check (csr_check.sh) into gpurun_out/<dir>
set -o pipefail
OUT=gpurun_out/${1:-pc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
bash tools/runs/csr_check.sh ${1:-pc}/csr
