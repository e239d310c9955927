#!/bin/bash
# Round 5 (k): the one-plane H = 256 stream-GEMM path (LN1 prologue, LN2 epilogue, 768 x 256 weight gradients over
# three column groups): LN / stream-GEMM tests, then C5 bf16 on the library GEMMs (TAGAN_SG_BF16_MAX_H=128) against
# the stream GEMMs (=256), interleaved x2, and a rocprofv3 kernel-stats pass of the stream-GEMM C5 step.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5k}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_sgemm_ln.py tests/test_gpu_sgemm.py -m gpu -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager --sub-records none"
for rep in 1 2; do
  for mh in 128 256; do
    TAGAN_SG_BF16_MAX_H=$mh timeout -k 10 400 python bench.py --config c5 --precision bf16 $B > $OUT/c5_${mh}_$rep.json 2> $OUT/c5_${mh}_$rep.err || { tail -20 $OUT/c5_${mh}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c5_${mh}_$rep.json'));print('c5 bf16 max_h=$mh', d['ms_per_step'], d.get('breakdown',{}).get('forward_ms'), d.get('breakdown',{}).get('backward_ms'))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAGAN_SG_BF16_MAX_H=256 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o run -- \
    python bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 \
    --precision bf16 --launch eager --sub-records none > $OUT/stats_c5.log 2>&1 || { tail -20 $OUT/stats_c5.log; exit 1; }
find $OUT/stats_c5 -name "*kernel_trace*" -delete
python tools/kstats.py $(find $OUT/stats_c5 -name "*kernel_stats.csv" | head -1) | sed -n 1,40p
