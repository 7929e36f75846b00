#!/bin/bash
# Interleaved A/B of libjpge variants (through gpurun): tools/ab_quick.sh ROUNDS name...
# (main = the tree's build, else jpgenc_amd/lib/var/<name>/); bench value + host CPU only.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
rounds=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq $rounds); do
  for n in "$@"; do
    lib=jpgenc_amd/lib/var/$n/libjpge.so
    [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
    JPGE_LIB=$lib timeout -k 10 200 python3 bench.py --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 2 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { tail -3 gpurun_out/ab/$n.err; exit 1; }
    echo "$n $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/$n.json').read().strip().splitlines()[-1]);print(d['value'], d['host_cpu']['cpus_used'], {k[:6]: round(v['avg_kernel_ms']*1e3,2) for k,v in d['stages_solo'].items()})")"
  done
done
