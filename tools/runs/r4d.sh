#!/bin/bash
# A/B of a compile-time switch of csrc/stream_gemm.hip (make variant NAME=ilv0 EXTRA=-DNT_INTERLEAVE=0) against the
# shipped library: the NT staging schedule; plus the stream-GEMM unit tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4d}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py -q --timeout 300 \
    --timeout-method thread > $OUT/unit.log 2>&1 || { tail -40 $OUT/unit.log; exit 1; }
tail -1 $OUT/unit.log
for lib in libtagan_hip.so libtagan_hip_ilv0.so; do
  TAGAN_LIB=$L/$lib SGEMM_PROBE_OUT=$OUT/probe_$lib.json timeout -k 10 300 python tools/sgemm_probe.py --H 128 \
      > $OUT/probe_$lib.log 2>&1 || { tail -20 $OUT/probe_$lib.log; exit 1; }
  TAGAN_LIB=$L/$lib timeout -k 10 300 python tools/tn_ab.py --H 128 >> $OUT/tn_ab.jsonl 2>&1 || { tail -20 $OUT/tn_ab.jsonl; exit 1; }
done
grep '^{' $OUT/tn_ab.jsonl
python - <<PY
import json
libs = ["libtagan_hip.so", "libtagan_hip_ilv0.so"]
d = {l: {c["case"]: c for c in json.load(open("$OUT/probe_%s.json" % l))["cases"]} for l in libs}
for k in d[libs[0]]:
    print("%-18s" % k, "  ".join("%s %8.1f" % (l.replace("libtagan_hip", "").replace(".so", "") or "main", d[l][k]["us_kernel"]) for l in libs))
PY
