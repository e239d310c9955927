#!/bin/bash
# PMC counters of the CSR builder kernels on one C4 snapshot (tools/csr_bench.py --configs c4), one pass per set.
set -o pipefail
OUT=gpurun_out/${1:-csrpmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/$OUT/p1 -o run -- python3 $R/tools/csr_bench.py --configs c4 --reps 1 > $R/$OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_WR -d $R/$OUT/p2 -o run -- python3 $R/tools/csr_bench.py --configs c4 --reps 1 > $R/$OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_EA0_WRREQ_sum -d $R/$OUT/p3 -o run -- python3 $R/tools/csr_bench.py --configs c4 --reps 1 > $R/$OUT/p3.log 2>&1 || exit 1
echo done
