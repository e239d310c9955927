# v6 backward register budget A/B at C2 / C4 / C1: default build (3 waves/SIMD) vs WPE_B=2 build vs v4
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-v6ab2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal_v6.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in c2 c4 c1; do
  for mode in "1 default" "1 tools/probes/lib_v6wpe2.so" "0 default"; do
    set -- $mode
    if [ "$2" = default ]; then unset TAGAN_LIB; else export TAGAN_LIB=$GRAFT_REPO_ROOT/$2; fi
    TAGAN_TATTN_V6=$1 timeout -k 10 200 python tools/tattn_kernels.py --config $cfg --reps 20 > $OUT/k.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    echo "$cfg V6=$1 $(cut -c1-250 $OUT/k.json)"
  done
done
