#!/bin/bash
# Interleaved A/B of environment settings on the single-image call (bench `latency` key):
#   tools/ab_latency.sh ROUNDS "A=1" "-" ...   ("-" = no extra setting)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
rounds=$1; shift
mkdir -p gpurun_out/abl
for r in $(seq $rounds); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    o=gpurun_out/abl/v$i
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python3 bench.py --frames 64 --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 --latency-calls 256 > $o.json 2> $o.err || { echo "== [$e] failed"; tail -3 $o.err; exit 1; }
    echo "[$e] $(python3 -c "
import json;d=json.loads(open('$o.json').read().strip().splitlines()[-1])
l=d['latency']['device_in_device_out']; print(l['median_ms'], l['p99_ms'], l['min_ms'])")"
  done
done
