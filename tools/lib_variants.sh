#!/bin/bash
# Build libjpge variants with extra -D flags on the HIP sources (diagnostic A/B runs):
#   tools/lib_variants.sh name "-DFOO=1 ..." [name "flags"] ...  (host and device sources alike)
#   -> jpgenc_amd/lib/var/<name>/libjpge.so (use with JPGE_LIB=...)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
while [ $# -ge 2 ]; do
  make -s -j8 BUILD=build/var_$1 LIBDIR=jpgenc_amd/lib/var/$1 HIPEXTRA="$2" jpgenc_amd/lib/var/$1/libjpge.so
  shift 2
done
