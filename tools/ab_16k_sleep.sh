#!/bin/bash
# 16384^2 pipeline: lane waits with and without the first long sleep.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for e in JPGE_FIRST_SLEEP=0 JPGE_FIRST_SLEEP=70 "JPGE_FIRST_SLEEP=0 JPGE_STATS_WGS=256 JPGE_LIB=jpgenc_amd/lib/var/mr/libjpge.so"; do
    env $e timeout -k 10 300 python3 bench.py --width 16384 --height 16384 --frames 16 --distinct 4 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/ab/x.json 2> gpurun_out/ab/x.err || { tail -3 gpurun_out/ab/x.err; exit 1; }
    echo "$e $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/x.json').read().strip().splitlines()[-1]);print(d['value'], d['host_cpu']['cpus_used'])")"
  done
done
