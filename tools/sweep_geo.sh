#!/bin/bash
# Edge-kernel variant sweep on one GPU (run through gpurun); results -> gpurun_out/sweep/geo.jsonl
set -e
mkdir -p gpurun_out/sweep
OUT=gpurun_out/sweep/geo.jsonl
run() { timeout -k 10 300 python tools/geo_kernels.py "$@" >> $OUT 2>> gpurun_out/sweep/geo.err; }
for lib in "" variants/libtagan_u2.so variants/libtagan_u8.so; do
  TAGAN_LIB=$lib run --config c2
done
for c in 32 64 256; do run --config c2 --chunk $c; done
run --config c2 --metric 6
run --config c4 --snapshots 4
TAGAN_LIB=variants/libtagan_u8.so run --config c4 --snapshots 4
run --config c4
