#!/bin/bash
# Per-thread host CPU of the 4K and batch1080 bench lines (through gpurun).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/tc
export JPGE_BENCH_THREADS=1
timeout -k 10 200 python3 bench.py --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 "$@" > gpurun_out/tc/a.json 2> gpurun_out/tc/a.err || { tail -3 gpurun_out/tc/a.err; exit 1; }
grep threads: gpurun_out/tc/a.err; python3 -c "import json;d=json.loads(open('gpurun_out/tc/a.json').read().strip().splitlines()[-1]);print(d['value'],d['host_cpu'])"
timeout -k 10 200 python3 bench.py --workload batch1080 --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/tc/b.json 2> gpurun_out/tc/b.err || { tail -3 gpurun_out/tc/b.err; exit 1; }
grep threads: gpurun_out/tc/b.err; python3 -c "import json;d=json.loads(open('gpurun_out/tc/b.json').read().strip().splitlines()[-1]);print(d['value'],d['host_cpu'])"
