#!/bin/bash
# Round 4: stream-GEMM unit tests (H = 64 / 128 / 256), the per-shape probe at H = 128 and 256, and SQ counter passes
# over the H = 128 probe.   bash tools/runs/r4b.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 300 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
SGEMM_PROBE_OUT=$OUT/probe_h128.json timeout -k 10 300 python tools/sgemm_probe.py --H 128 > $OUT/probe_h128.log 2>&1 \
    || { tail -20 $OUT/probe_h128.log; exit 1; }
SGEMM_PROBE_OUT=$OUT/probe_h256.json timeout -k 10 300 python tools/sgemm_probe.py --H 256 --M 1600000 \
    > $OUT/probe_h256.log 2>&1 || { tail -20 $OUT/probe_h256.log; exit 1; }
python - <<PY
import json
for h in ("h128", "h256"):
    d = json.load(open("$OUT/probe_%s.json" % h))
    for c in d["cases"]:
        print(h, "%-18s" % c["case"], "kernel %8.1f us  torch %8.1f us  %6.2f TB/s  %7.1f TF/s" %
              (c["us_kernel"], c["us_torch"], c["TBps_kernel"], c["TFps_kernel"]))
PY
bash tools/sq_counters.sh ${1:-r4b} python tools/sgemm_probe.py --H 128 --M 320000 > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
cp gpurun_out/sq_${1:-r4b}/table.txt $OUT/pmc_table.txt
grep -A 20 "k_sgemm" $OUT/pmc_table.txt | head -120
# the round-4 tests added beside the GEMM work: C5-geometry two-rank shard (gloo on one GPU), C3/C5-geometry whole
# model against the fp64 oracle
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py::test_sharded_hip_matches_unsharded_c5_geometry \
    "tests/test_gpu_fullsize.py::test_geometry_whole_model_vs_oracle" -v --timeout 850 --timeout-method thread \
    > $OUT/new_tests.log 2>&1; echo "new tests rc=$?"; grep -E "PASS|FAIL|Error|error" $OUT/new_tests.log | head -20
