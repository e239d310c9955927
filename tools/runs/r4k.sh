#!/bin/bash
# Temporal kernels with and without dropout at the C5 / C3 / C2 shapes (what the counter-hash mask costs), SQ counter
# passes of the C5 kernels (plus MFMA busy cycles and the clock), and the CSR side-stream A/B (the shipped library
# against libtagan_hip_noside.so: big-bucket kernels on the caller's stream), in-step and standalone.
#   bash tools/runs/r4k.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4k}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
for c in c5 c3 c2; do
  for p in 0.1 0; do
    timeout -k 10 200 python tools/tattn_kernels.py --config $c --p $p --reps 5 > $OUT/tattn_${c}_p$p.json 2>&1 \
        || { tail -5 $OUT/tattn_${c}_p$p.json; exit 1; }
    echo "$c p=$p $(tail -1 $OUT/tattn_${c}_p$p.json)"
  done
done
for rep in 1 2; do
  for lib in libtagan_hip.so libtagan_hip_noside.so; do
    TAGAN_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-c1 \
        > $OUT/bench_${lib}_$rep.json 2> $OUT/bench_${lib}_$rep.err || { tail -20 $OUT/bench_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d['alt_precision']['ms_per_step'], d['breakdown']['csr_build_ms'])"
    TAGAN_LIB=$L/$lib timeout -k 10 200 python tools/csr_bench.py --configs c2,c4 --reps 10 > $OUT/csr_${lib}_$rep.json 2>&1 \
        || { tail -5 $OUT/csr_${lib}_$rep.json; exit 1; }
    tail -2 $OUT/csr_${lib}_$rep.json
  done
done
bash tools/sq_counters.sh ${1:-r4k}_c5 python tools/tattn_kernels.py --config c5 --reps 1 || exit 1
cat gpurun_out/sq_${1:-r4k}_c5/table.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU \
    --kernel-trace --output-format csv -d $OUT/mfma_c5 -- python tools/tattn_kernels.py --config c5 --reps 1 \
    > $OUT/mfma_c5.log 2>&1 || { tail -5 $OUT/mfma_c5.log; exit 1; }
find $OUT/mfma_c5 -name "*kernel_trace*" -delete
python tools/pmc_table.py $OUT/mfma_c5 || true
