#!/bin/bash
# Interleaved A/B of environment settings (through gpurun): tools/ab_env.sh ROUNDS "A=1 B=2" "A=0" ...
# ("-" = no extra setting).  Prints the bench value, host CPU, solo and in-situ kernel times.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
rounds=$1; shift
mkdir -p gpurun_out/abe
for r in $(seq $rounds); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    o=gpurun_out/abe/v$i
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python3 bench.py ${AB_ARGS:---frames 1536 --steps 8} --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 2 > $o.json 2> $o.err || { echo "== [$e] failed"; tail -3 $o.err; exit 1; }
    echo "[$e] $(python3 -c "
import json;d=json.loads(open('$o.json').read().strip().splitlines()[-1])
f=lambda s:{k[:6]: round(v['avg_kernel_ms']*1e3,2) for k,v in (d.get(s) or {}).items()}
print(d['value'], d['host_cpu']['cpus_used'], 'solo', f('stages_solo'), 'single', f('stages_solo_single_frame'), 'situ', f('stages'))")"
  done
done
