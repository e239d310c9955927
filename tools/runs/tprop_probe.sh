set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tprop
for cfg in c2 c4; do
  for bi in 0 1; do
    timeout -k 10 300 python tools/tprop_probe.py --config $cfg --bidirectional $bi --reps 5 || exit 1
  done
done | tee gpurun_out/tprop/probe.jsonl
