#!/bin/bash
# Round 5 (c): the fused LN2 backward + out-projection gradients (tagan_ln2_bwd_out) and the forced watchdog race with
# the fix: their GPU tests and the backward parity suites; the same-process step A/B with and without "ln2bwd"
# (tools/ab_step.py, fp32 and bf16); the per-product probe; SQ / MFMA counters of the fp32 QKV forward (LDS-DMA
# k_sgemm_ntg against the register-staged k_sgemm_nt).   bash tools/runs/r5c.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5c}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/temporal-asymmetric-graph-attention-network_amd
TAGAN_PARITY_LOG=$OUT/parity_errors.json timeout -k 10 700 python -u -m pytest tests/test_gpu_sgemm_ln.py \
    tests/test_gpu_rccl.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_graph.py \
    tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_dp.py -m gpu -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/ab_step.py --precision fp32 in+out in+out+ln2bwd > $OUT/ab_fp32.log 2>&1 || { tail -20 $OUT/ab_fp32.log; exit 1; }
grep -i median $OUT/ab_fp32.log
timeout -k 10 300 python tools/ab_step.py --precision bf16 in+out+bwd all > $OUT/ab_bf16.log 2>&1 || { tail -20 $OUT/ab_bf16.log; exit 1; }
grep -i median $OUT/ab_bf16.log
TAGAN_LIB=$L/libtagan_hip.so timeout -k 10 300 python tools/sgemm_probe.py --planes 3,1 \
    --cases qkv_fwd,qkv_fwd_ln,dc,dw_o,ln2_bwd_out > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
python -c "
import json
for l in open('$OUT/probe.log'):
    if l.startswith('{'):
        c = json.loads(l); print('%-22s %7.1f us %6.3f TB/s' % (c['case'], c['us_kernel'], c['TBps_kernel']))"
for lib in libtagan_hip.so libtagan_hip_noglds.so; do
  TAGAN_LIB=$L/$lib timeout -k 10 200 bash tools/sq_counters.sh qkv_$lib python tools/sgemm_probe.py --planes 3 \
      --cases qkv_fwd_ln || { echo "sq pass failed ($lib)"; exit 1; }
  TAGAN_LIB=$L/$lib timeout -k 10 200 bash tools/runs/mfma_pmc.sh qkv_$lib python tools/sgemm_probe.py --planes 3 \
      --cases qkv_fwd_ln > /dev/null || { echo "mfma pass failed ($lib)"; exit 1; }
  echo "== $lib"; python tools/pmc_table.py gpurun_out/sq_qkv_$lib sgemm_nt; python tools/pmc_table.py gpurun_out/mp_qkv_$lib sgemm_nt
done
