#!/bin/bash
# Diag build's per-workgroup phase stamps of one 4K frame (1 lane).  -> gpurun_out/st_<tag>/
set -u
cd ${GRAFT_REPO_ROOT:-.}
o=gpurun_out/st_$1; mkdir -p $o
JPGE_LIB=jpgenc_amd/lib/diag/libjpge.so JPGE_STAMPS_FILE=$o/stamps.bin timeout -k 10 120 \
  python3 tools/prof_frame.py --iters 3 > $o/stamps.log 2>&1 || { tail -5 $o/stamps.log; exit 1; }
python3 tools/stamps.py $o/stamps.bin > $o/stamps.txt 2>&1; cat $o/stamps.txt
