#!/bin/bash
# CSR builder parity + C2 bench (fp32 headline) after a CSR change.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/csr
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "csr or golden" \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $OUT/bench.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], d['breakdown']['csr_build_ms'], d['alt_precision']['ms_per_step'])"
