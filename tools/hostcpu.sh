#!/bin/bash
# Host CPU per GPU (diagnostic): the 4K bench with per-thread CPU and thread-state
# samples under a few host settings.  tools/hostcpu.sh <tag> ["ENV=.. ENV=.." ...]
set -u
cd ${GRAFT_REPO_ROOT:-.}
tag=$1; shift
o=gpurun_out/hc_$tag; mkdir -p $o
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs JPGE_BENCH_THREADS=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --d2h-steps 0 --steps 10 --solo-batches 1 > $o/b$i.json 2> $o/b$i.err || { tail -5 $o/b$i.err; exit 1; }
  echo "== $envs"; python3 -c "
import json,sys; d=json.loads([l for l in open('$o/b$i.json') if l.startswith('{')][-1]); print('value', d['value'], 'host_cpu', d['host_cpu'])"
  grep -E "^threads|^sampler" $o/b$i.err | cut -c1-400
done
true
