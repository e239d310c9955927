# v6 (head-group slabs) vs v4: parity, then kernel times at C2 / C4 / C1 for GH = 4, 2 and v4
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v6ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_temporal_v6.py \
    tests/test_gpu_temporal_v4.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for cfg in c2 c4; do
  for mode in "1 4" "1 2" "0 4"; do
    set -- $mode
    TAGAN_TATTN_V6=$1 TAGAN_V6_GH=$2 timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    echo "$cfg V6=$1 GH=$2 $(cut -c1-260 $OUT/k.json)"
  done
done
