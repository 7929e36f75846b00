#!/bin/bash
# bench.py value per environment setting: tools/env_sweep.sh "JPGE_LOOKAHEAD=3 JPGE_DRAIN_LAG=1" ...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for e in "$@"; do
  env $e timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/es.json 2> gpurun_out/es.err || { echo "== $e failed"; tail -3 gpurun_out/es.err; continue; }
  echo "== $e: $(python3 -c "import json;d=json.loads(open('gpurun_out/es.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d.get('host_cpu'))")"
done
