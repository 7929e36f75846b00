#!/bin/bash
# bench.py value per (hardware queues, lanes): tools/hwq_sweep.sh "4 4" "8 8" ...
# (GPU_MAX_HW_QUEUES: HIP's hardware queues per process, 4 by default)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for c in "$@"; do
  set -- $c
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python3 bench.py --lanes $2 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/hq.json 2> gpurun_out/hq.err || { echo "== $c failed"; tail -3 gpurun_out/hq.err; exit 1; }
  echo "== queues $1 lanes $2: $(python3 -c "import json;d=json.loads(open('gpurun_out/hq.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['lanes'])")"
done
