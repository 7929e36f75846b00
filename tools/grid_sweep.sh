#!/bin/bash
# bench.py value per (library variant, K2 workgroups, entropy workgroups):
#   tools/grid_sweep.sh main:0:0 t8:0:256:6 ...   (0 = the library's default; "main" = the product;
#   an optional 4th field: lanes)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for p in "$@"; do
  IFS=: read -r n k2 k3 ln <<< "$p"
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib JPGE_STATS_WGS=$k2 JPGE_ENTROPY_WGS=$k3 timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 --lanes ${ln:-0} > gpurun_out/gs.json 2> gpurun_out/gs.err || exit 1
  echo "== $n k2 $k2 k3 $k3 lanes ${ln:-0}: $(python3 -c "import json;d=json.loads(open('gpurun_out/gs.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
