#!/bin/bash
# 16384^2 bench value per libjpge variant: tools/ab_16k.sh name...  (main = the working tree's library)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
A="--width 16384 --height 16384 --frames 16 --distinct 2 --steps 8 --warmup 1 --d2h-steps 0 --solo-batches 0 --no-verify --no-cpu-baseline"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py $A > gpurun_out/a16_$n.json 2> gpurun_out/a16_$n.err || { tail -3 gpurun_out/a16_$n.err; exit 1; }
  echo "== 16k $n: $(python3 -c "import json;d=json.loads(open('gpurun_out/a16_$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
