#!/bin/bash
# Full validation of the temporal-dropout / keep-cache / pipelined-backward tree: GPU suite (parity log), the parity
# subset on the bounds-check build, the default bench line, C2 kernel stats (fp32, bf16), SQ counters of the C5
# temporal kernels.   bash tools/runs/r4n.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4n}
mkdir -p $OUT
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
TAGAN_LIB=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_debug.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membank.py tests/test_gpu_ingest.py \
    tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_v5.py tests/test_gpu_sgemm.py tests/test_gpu_debug.py -m gpu \
    -x -q --timeout 300 --timeout-method thread > $OUT/debug_tests.log 2>&1 || { tail -40 $OUT/debug_tests.log; exit 1; }
tail -1 $OUT/debug_tests.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['alt_precision']['ms_per_step'], d['roofline']['frac'], d['temporal_kernels'][1]['frac_bwd'], d['breakdown']['csr_build_ms'])"
bash tools/runs/c2_prof2.sh ${1:-r4n} > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
grep -v "^|" $OUT/prof.log | head -30
bash tools/sq_counters.sh ${1:-r4n}_c5 python tools/tattn_kernels.py --config c5 --reps 1 || exit 1
grep -A19 "k_tattn" gpurun_out/sq_${1:-r4n}_c5/table.txt | head -40
