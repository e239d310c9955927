#!/bin/bash
# Build libtagan_hip.so variants with temporal v4 knobs into variants/ (git-ignored) and report the
# v4 kernels' register use.  Usage: bash tools/runs/build_v4_variants.sh "name:FLAGS" ...
set -e
cd "$(dirname "$0")/../.."
CS=temporal-asymmetric-graph-attention-network_amd/csrc
mkdir -p variants
for spec in "$@"; do
  name=${spec%%:*}
  flags=${spec#*:}
  make -s -C $CS -j8 BUILD=build_$name OUT=../../variants/$name.so EXTRA="$flags" >/dev/null
  echo "== $name ($flags)"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $flags -c $CS/temporal_attn.hip \
      -o /tmp/ta_$name.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A12 "_v4ILi2ELi1EfE" \
      | grep -E "Function Name|VGPRs:|AGPRs|VGPRs Spill|Occupancy" | sed 's/.*remark: //; s/ \[-Rpass.*//; s/_ZN5tagan12_GLOBAL__N_114//' \
      | paste - - - - -
done
