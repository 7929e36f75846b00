#!/bin/bash
# K2 alone (the bench's solo pass) per statistics grid (JPGE_STATS_WGS also sets the pipeline's).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/k2s
for r in 1 2; do
  for w in 768 512 384 256; do
    JPGE_STATS_WGS=$w timeout -k 10 200 python3 bench.py --frames 256 --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 4 > gpurun_out/k2s/a.json 2> gpurun_out/k2s/a.err || { tail -3 gpurun_out/k2s/a.err; exit 1; }
    echo "$w: $(python3 -c "import json;d=json.loads(open('gpurun_out/k2s/a.json').read().strip().splitlines()[-1]);v=d['stages_solo']['stats_kernel'];print(round(v['avg_kernel_ms']*1e3,2), v['frac'])")"
  done
done
