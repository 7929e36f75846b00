#!/bin/bash
# D2H-inclusive figure (bench.py's d2h: .jpg bytes landing in pinned host memory) per
# libjpge variant: tools/ab_d2h.sh name...  (main = the working tree's library)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 10 --no-verify --solo-batches 0 > gpurun_out/d2h_$n.json 2> gpurun_out/d2h_$n.err || exit 1
  echo "== d2h $n: $(python3 -c "import json;d=json.loads(open('gpurun_out/d2h_$n.json').read().strip().splitlines()[-1]);print(d['d2h'])")"
done
