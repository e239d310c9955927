# C2 backward: v6 forced (TAGAN_TATTN_V6=2) vs v4, GH 4 / 2 / 8, after parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v6ab4}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal_v6.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for mode in "2 4" "2 2" "2 8" "0 4"; do
  set -- $mode
  TAGAN_TATTN_V6=$1 TAGAN_V6_GH=$2 timeout -k 10 200 python tools/tattn_kernels.py --config c2 --reps 30 > $OUT/k.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
  echo "c2 V6=$1 GH=$2 $(cut -c1-200 $OUT/k.json)"
done
done
