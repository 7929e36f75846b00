#!/bin/bash
# Build K1 micro-bench variants of the product fdct.hip with extra -D flags (diagnostic).
#   tools/k1_variants.sh name "-DFOO=1 ..." [name "flags"] ...
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/build/k1"
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off $2 -I"$R/jpgenc_amd/csrc" -I"$R/include" \
    -o "$R/build/k1/k1_$1" "$R/tools/k1_micro.cpp" "$R/jpgenc_amd/csrc/fdct.hip" &
  shift 2
done
wait
