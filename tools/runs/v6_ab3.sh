# v6 group width A/B (forward at C2, both at C4) + parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v6ab3}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal_v6.py tests/test_gpu_temporal_v4.py tests/test_gpu_temporal_T.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in c2 c4; do
  for mode in "1 8" "1 4" "1 2" "0 4"; do
    set -- $mode
    TAGAN_TATTN_V6=$1 TAGAN_V6_GH=$2 timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    echo "$cfg V6=$1 GH=$2 $(cut -c1-230 $OUT/k.json)"
  done
done
