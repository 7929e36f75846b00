#!/bin/bash
# K2 LDS/occupancy sensitivity (through gpurun): main vs K2_NZCAP=4096 (36 KB LDS, outputs
# invalid on overflow; --no-verify) at 2 and 3 statistics workgroups per CU, and 4 per CU.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
run() {  # name lib env...
  n=$1; lib=$2; shift 2
  env JPGE_LIB=$lib "$@" timeout -k 10 300 python3 bench.py --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { tail -3 gpurun_out/ab/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/$n.json').read().strip().splitlines()[-1]);print(d['value'])")"
}
for r in 1 2; do
  run main jpgenc_amd/lib/libjpge.so
  run main768 jpgenc_amd/lib/libjpge.so JPGE_STATS_WGS=768
  run nz512 jpgenc_amd/lib/var/nz/libjpge.so
  run nz768 jpgenc_amd/lib/var/nz/libjpge.so JPGE_STATS_WGS=768
  run nz3_1024 jpgenc_amd/lib/var/nz3/libjpge.so JPGE_STATS_WGS=1024
done
