#!/bin/bash
# bench.py value per K2 grid size (JPGE_STATS_WGS) and lane count
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for l in ${LANES:-4 8}; do
  for w in ${WGS:-0 256 384}; do
    JPGE_STATS_WGS=$w timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --lanes $l > gpurun_out/sw_$l_$w.json 2>gpurun_out/sw.err || exit 1
    echo "lanes $l wgs $w: $(python3 -c "import json;d=json.loads(open('gpurun_out/sw_$l_$w.json').read().strip().splitlines()[-1]);s=d['stages'];print(d['value'],[round(s[k]['avg_kernel_ms']*1000,1) for k in s])")"
  done
done
