# Temporal kernel cost split at C2: dropout on/off, v4 vs v5 (TT = 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-tprobe}
mkdir -p $OUT
for p in 0.1 0.0; do
  for v in 1 2; do
    TAGAN_TATTN_V5=$v timeout -k 10 120 python tools/tattn_kernels.py --config c2 --p $p --reps 30 > $OUT/c2_p${p}_v5$v.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    echo "p=$p V5=$v $(cut -c1-330 $OUT/c2_p${p}_v5$v.json)"
  done
done
