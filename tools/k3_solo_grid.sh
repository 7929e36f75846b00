#!/bin/bash
# Entropy kernels alone (the bench's solo pass) per grid (JPGE_ENTROPY_WGS also sets the pipeline's).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/k3s
for r in 1 2; do
  for w in 512 256 384 768 1024; do
    JPGE_ENTROPY_WGS=$w timeout -k 10 200 python3 bench.py --frames 256 --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 4 > gpurun_out/k3s/a.json 2> gpurun_out/k3s/a.err || { tail -3 gpurun_out/k3s/a.err; exit 1; }
    echo "$w: $(python3 -c "import json;d=json.loads(open('gpurun_out/k3s/a.json').read().strip().splitlines()[-1]);s=d['stages_solo'];print({k[:12]: round(v['avg_kernel_ms']*1e3,2) for k,v in s.items()})")"
  done
done
