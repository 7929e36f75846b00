#!/bin/bash
# Interleaved A/B of libjpge variants on one bench workload (through gpurun):
#   tools/ab_workload.sh ROUNDS "bench args" name...   (main = the tree's build, else jpgenc_amd/lib/var/<name>/)
# prints the bench value and the host CPU per run.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
rounds=$1; shift
args=$1; shift
mkdir -p gpurun_out/abw
for r in $(seq $rounds); do
  for n in "$@"; do
    lib=jpgenc_amd/lib/var/$n/libjpge.so
    [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
    JPGE_LIB=$lib timeout -k 10 200 python3 bench.py $args --no-cpu-baseline --no-verify --solo-batches 0 --d2h-steps 0 --latency-calls 0 > gpurun_out/abw/$n.$r.json 2> gpurun_out/abw/$n.$r.err || { tail -3 gpurun_out/abw/$n.$r.err; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/abw/$n.$r.json') if l.startswith('{')][-1])
h=d.get('host_cpu') or {}
print('$n', d['value'], 'ms/step', d['ms_per_step'], 'cpus', h.get('cpus_used'), 'rank', d.get('rank_cpus'))"
  done
done
