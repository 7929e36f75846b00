#!/bin/bash
# 16384^2 pipeline: statistics grid 512 (main) vs 256 with 256-tile runs (var/mr).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in "main jpgenc_amd/lib/libjpge.so" "mr256 jpgenc_amd/lib/var/mr/libjpge.so JPGE_STATS_WGS=256"; do
    set -- $v; n=$1; lib=$2; shift 2
    env JPGE_LIB=$lib "$@" timeout -k 10 300 python3 bench.py --width 16384 --height 16384 --frames 16 --distinct 4 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { tail -3 gpurun_out/ab/$n.err; exit 1; }
    echo "$n $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/$n.json').read().strip().splitlines()[-1]);print(d['value'])")"
  done
done
