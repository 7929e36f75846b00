#!/bin/bash
# A/B timing of libjpge variants on the single-frame loop (16 distinct 4K frames):
#   tools/ab_frames.sh name... (jpgenc_amd/lib/var/<name>/libjpge.so; "main" = the product)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  for rep in 1 2; do
    echo "== $n: $(JPGE_LIB=$lib timeout -k 10 120 python3 tools/prof_frame.py --frames 16 --iters 64 2>&1 | tail -1)"
  done
done
