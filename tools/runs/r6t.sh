#!/bin/bash
# Round 6 (t): C2 temporal backward, v4 against the v6 head-group slabs (TAGAN_TATTN_V6=2 forces v6's backward) at
# GH = 2 / 4 / 8, fp32 and bf16, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r6t}
mkdir -p $OUT
for r in 1 2; do
  for v in v4 g2 g4 g8; do
    case $v in v4) E="TAGAN_TATTN_V6=1";; g2) E="TAGAN_TATTN_V6=2 TAGAN_V6_GH=2";; g4) E="TAGAN_TATTN_V6=2 TAGAN_V6_GH=4";; g8) E="TAGAN_TATTN_V6=2 TAGAN_V6_GH=8";; esac
    for b in "" "--bf16"; do
      env $E timeout -k 10 120 python tools/tattn_kernels.py --config c2 --reps 20 $b > $OUT/t_$v$b.$r.json 2>&1 || { tail -5 $OUT/t_$v$b.$r.json; exit 1; }
      echo "$v $b run $r: $(tail -1 $OUT/t_$v$b.$r.json | cut -c1-400)"
    done
  done
done
