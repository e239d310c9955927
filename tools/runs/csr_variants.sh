#!/bin/bash
# CSR builder variants (variants/libt*.so built with -DTAGAN_CSR_TARGET=...): bit-exact tests + timing each
set -o pipefail
OUT=gpurun_out/${1:-csrvar}
mkdir -p $OUT
for L in "" variants/libt1024.so variants/libt1536.so; do
  tag=$(basename "${L:-default}")
  TAGAN_LIB=${L:+$PWD/$L} timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k csr -x -q --timeout 120 --timeout-method thread > $OUT/t_$tag.log 2>&1 || { tail -30 $OUT/t_$tag.log; exit 1; }
  echo "$tag: $(tail -1 $OUT/t_$tag.log)"
  TAGAN_LIB=${L:+$PWD/$L} timeout -k 10 300 python -u tools/csr_bench.py --configs c2,c4 > $OUT/b_$tag.log 2>&1 || { tail -30 $OUT/b_$tag.log; exit 1; }
  grep build_ms $OUT/b_$tag.log
done
