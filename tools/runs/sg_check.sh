#!/bin/bash
# stream-GEMM tests, then the C2 bench with and without the stream GEMMs (A/B, same box), then the whole GPU suite
set -o pipefail
OUT=gpurun_out/${1:-sgc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py -x -q --timeout 120 --timeout-method thread > $OUT/sgemm_tests.log 2>&1 || { tail -30 $OUT/sgemm_tests.log; exit 1; }
tail -2 $OUT/sgemm_tests.log
for v in 1 0 1; do
  TAGAN_SGEMM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 > $OUT/bench_sg$v.json 2> $OUT/bench_sg$v.err || { tail -20 $OUT/bench_sg$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_sg$v.json'));print('sgemm=$v', d['ms_per_step'], d.get('alt_precision',{}).get('ms_per_step'))"
done
bash tools/runs/gpu_suite.sh ${1:-sgc}
