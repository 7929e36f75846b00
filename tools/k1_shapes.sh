#!/bin/bash
# K1 alone (the bench's solo pass) per frame size and subsampling: 4K 4:2:0 and 4:4:4
# (4-wave shape, 4 per CU) and 16384^2 (whole-CU shape).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/k1s
for r in 1 2; do
  for size in "--subsampling 420" "--subsampling 444" "--width 16384 --height 16384 --frames 16 --distinct 4"; do
    timeout -k 10 200 python3 bench.py --frames 256 --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 4 $size > gpurun_out/k1s/a.json 2> gpurun_out/k1s/a.err || { tail -3 gpurun_out/k1s/a.err; exit 1; }
    echo "$size: $(python3 -c "import json;d=json.loads(open('gpurun_out/k1s/a.json').read().strip().splitlines()[-1]);v=d['stages_solo']['fdct_kernel'];print(round(v['avg_kernel_ms']*1e3,2), v['frac'], d['value'])")"
  done
done
