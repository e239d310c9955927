#!/bin/bash
# A/B of temporal v4 build knobs (TAGAN_V4_*): parity tests on the default build, then kernel timings
# of each variant library under variants/ (built on the CPU host by tools/runs/build_v4_variants.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v4v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal_v4.py \
    tests/test_gpu_temporal_T.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for lib in default variants/*.so; do
    name=$(basename $lib .so)
    for cfg in c2 c4; do
      if [ $lib = default ]; then
        timeout -k 10 120 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>/dev/null || exit 1
      else
        TAGAN_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>/dev/null || exit 1
      fi
      python -c "import json;d=json.load(open('$OUT/k.json'));print('%-14s %s fwd %.4f bwd %.4f' % ('$name', '$cfg', d['ms_fwd'], d['ms_bwd']))"
    done
  done
done
