#!/bin/bash
# One diagnostic GPU call: solo kernel durations (rocprof), SQ counters, and the
# diag build's per-workgroup phase stamps of one 4K frame.
#   tools/diag_round.sh <tag>   ->  gpurun_out/diag_<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
tag=$1
out=gpurun_out/diag_$tag
mkdir -p "$out"
bash tools/prof_kernels.sh "$tag" > "$out/kernels.txt" 2>&1 || { cat "$out/kernels.txt"; exit 1; }
cat "$out/kernels.txt"
JPGE_LIB=jpgenc_amd/lib/diag/libjpge.so JPGE_STAMPS_FILE=$out/stamps.bin timeout -k 10 120 \
  python3 tools/prof_frame.py --iters 3 > "$out/stamps.log" 2>&1 || { tail -5 "$out/stamps.log"; exit 1; }
python3 tools/stamps.py "$out/stamps.bin" > "$out/stamps.txt" 2>&1; cat "$out/stamps.txt"
bash tools/pmc_sq.sh "$tag" --iters 8 > "$out/sq.txt" 2>&1 || { tail -5 "$out/sq.txt"; exit 1; }
cat "$out/sq.txt"
