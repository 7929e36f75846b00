#!/bin/bash
# Host CPU vs throughput per lane-wait setting (through gpurun), interleaved so box drift
# spreads over the variants:  tools/sleep_sweep.sh "JPGE_FIRST_SLEEP=0" "JPGE_FIRST_SLEEP=70" ...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ss
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 200 python3 bench.py --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/ss/a.json 2> gpurun_out/ss/a.err || { echo "== $e failed"; tail -3 gpurun_out/ss/a.err; exit 1; }
    echo "4K    $e: $(python3 -c "import json;d=json.loads(open('gpurun_out/ss/a.json').read().strip().splitlines()[-1]);print(d['value'],d['host_cpu']['cpus_used'])")"
    env $e timeout -k 10 200 python3 bench.py --workload batch1080 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ss/b.json 2> gpurun_out/ss/b.err || { echo "== $e failed"; tail -3 gpurun_out/ss/b.err; exit 1; }
    echo "1080b $e: $(python3 -c "import json;d=json.loads(open('gpurun_out/ss/b.json').read().strip().splitlines()[-1]);print(d['value'],d['host_cpu']['cpus_used'])")"
  done
done
