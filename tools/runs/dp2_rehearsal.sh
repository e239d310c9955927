#!/bin/bash
# two ranks on one GPU over gloo (bench.py's rehearsal knobs): the N > 1 flow end to end, exit status included
set -o pipefail
OUT=gpurun_out/${1:-dp2r}
mkdir -p $OUT
TAGAN_BENCH_BACKEND=gloo TAGAN_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --sub-records ${2:-none} \
    > $OUT/b.json 2> $OUT/b.err
rc=$?
echo "rc=$rc"
tail -c 1500 $OUT/b.json
exit $rc
