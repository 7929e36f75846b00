#!/bin/bash
# A/B of libjpge variants on one box: tools/ab_libs.sh ROUNDS name... (main = the tree's
# build, else jpgenc_amd/lib/var/<name>/): bench value and solo kernel times per run.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
rounds=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq $rounds); do
  for n in "$@"; do
    lib=jpgenc_amd/lib/var/$n/libjpge.so
    [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
    JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 2 > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err || { tail -3 gpurun_out/ab/$n.$r.err; exit 1; }
    python3 - gpurun_out/ab/$n.$r.json $n <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
so = d.get("stages_solo") or {}
print(f"{sys.argv[2]:10s} {d['value']:9.1f}  solo " + " ".join(f"{k.split('_')[0][:5]}{'' if 'kernel' not in k else k.split('_')[1][:4]}={v['avg_kernel_ms']*1e3:.2f}" for k, v in so.items()), "cpu", d["host_cpu"]["cpus_used"] if d.get("host_cpu") else "")
PY
  done
done
true
