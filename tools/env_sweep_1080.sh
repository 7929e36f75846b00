#!/bin/bash
# batch1080 (config 4) bench value per environment setting: tools/env_sweep_1080.sh "JPGE_STATS_WGS=190" ...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for e in "$@"; do
  env $e timeout -k 10 300 python3 bench.py --workload batch1080 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/e1080.json 2> gpurun_out/e1080.err || { echo "== $e failed"; tail -3 gpurun_out/e1080.err; exit 1; }
  echo "== $e: $(python3 -c "import json;d=json.loads(open('gpurun_out/e1080.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_cpu']['cpus_used'])")"
done
