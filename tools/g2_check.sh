#!/bin/bash
# 2 ranks of bench.py on this box per libjpge variant: exit status and value
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_DEBUG=1 JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --gpus 2 --steps 2 --warmup 1 --d2h-steps 0 --solo-batches 0 --no-verify --no-cpu-baseline > gpurun_out/g2_$n.json 2> gpurun_out/g2_$n.err
  echo "== $n rc=$? $(tail -c 120 gpurun_out/g2_$n.json | tr -d '\n' | head -c 120) $(grep -o 'JPGE_E_[A-Z]*' gpurun_out/g2_$n.err | head -1)"
done
