#!/bin/bash
# Build the K1 micro-benchmark against one or more fdct.hip variants (diagnostic).
#   tools/k1_micro.sh out_dir [variant.hip ...]   (default: the product's fdct.hip)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/build/k1}
shift || true
mkdir -p "$OUT"
srcs=("$@")
[ ${#srcs[@]} -eq 0 ] && srcs=("$R/jpgenc_amd/csrc/fdct.hip")
for s in "${srcs[@]}"; do
  n=$(basename "$s" .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$R/jpgenc_amd/csrc" -I"$R/include" \
    -o "$OUT/k1_$n" "$R/tools/k1_micro.cpp" "$s"
done
