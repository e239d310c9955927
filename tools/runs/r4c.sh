#!/bin/bash
# TN A/B (k_sgemm_tn2 vs k_sgemm_tn) at H = 128 / 256 + the stream-GEMM unit tests.   bash tools/runs/r4c.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 300 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
timeout -k 10 300 python tools/tn_ab.py --H 128 > $OUT/tn_ab_h128.jsonl 2>&1 || { tail -20 $OUT/tn_ab_h128.jsonl; exit 1; }
cat $OUT/tn_ab_h128.jsonl
timeout -k 10 300 python tools/tn_ab.py --H 256 --M 1600000 > $OUT/tn_ab_h256.jsonl 2>&1 || { tail -20 $OUT/tn_ab_h256.jsonl; exit 1; }
cat $OUT/tn_ab_h256.jsonl
# NT staging order A/B: the shipped library (stash first) against the round-3 order (make variant NAME=ntold)
SGEMM_PROBE_OUT=$OUT/probe_new.json timeout -k 10 300 python tools/sgemm_probe.py --H 128 > $OUT/probe_new.log 2>&1 || { tail -20 $OUT/probe_new.log; exit 1; }
TAGAN_LIB=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_ntold.so SGEMM_PROBE_OUT=$OUT/probe_old.json \
    timeout -k 10 300 python tools/sgemm_probe.py --H 128 > $OUT/probe_old.log 2>&1 || { tail -20 $OUT/probe_old.log; exit 1; }
python - <<PY
import json
a = {c["case"]: c for c in json.load(open("$OUT/probe_new.json"))["cases"]}
b = {c["case"]: c for c in json.load(open("$OUT/probe_old.json"))["cases"]}
for k in a:
    print("%-18s new %8.1f us  old %8.1f us" % (k, a[k]["us_kernel"], b[k]["us_kernel"]))
PY
