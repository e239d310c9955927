#!/bin/bash
# Round 6 (l): ping-pong NT default (plain / split-K only) vs no-pp variant at C3 (H = 256 split-K QKV dX), the
# stream-GEMM tests, the captured sharded-step RCCL case and the sharded GPU tests, and a one-GPU c5_shard
# sub-record rehearsal at reduced snapshot size (graph launch expected).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6l}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_sgemm_ln.py tests/test_gpu_rccl.py tests/test_gpu_sharded.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-c1 --no-roofline --no-alt-precision --sub-records c5_shard --c5-shard-size 4000,40000 --steps 3 --warmup 1 > $OUT/c5shard.json 2> $OUT/c5shard.err || { tail -20 $OUT/c5shard.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5shard.json'));r=d['c5_shard'];print('c5_shard rehearsal', r['launch'], r.get('launch_trial'), r['ms_per_step'], r['exchange_ms_per_step'])"
for r in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_nopp.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 500 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-alt-precision --no-c1 --launch eager > $OUT/c3_$lib.$r.json 2> $OUT/c3_$lib.$r.err || { tail -20 $OUT/c3_$lib.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c3_$lib.$r.json'));print('c3 $lib $r', d['ms_per_step'])"
  done
done
