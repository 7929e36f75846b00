#!/bin/bash
# batch1080 (config 4) under settings: tools/sweep_1080.sh "ENV=.. --lanes N" ...
# (each argument: environment assignments and bench flags; "-" = defaults)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s1080
i=0
for spec in "$@"; do
  i=$((i + 1))
  envs=(); flags=()
  for w in $spec; do
    case "$w" in
      -) ;;
      *=*) envs+=("$w") ;;
      *) flags+=("$w") ;;
    esac
  done
  o=gpurun_out/s1080/v$i
  env "${envs[@]}" timeout -k 10 200 python3 bench.py --workload batch1080 ${S1080_ARGS:---steps 30 --warmup 3} --no-cpu-baseline "${flags[@]}" > $o.json 2> $o.err || { echo "== [$spec] failed"; tail -3 $o.err; exit 1; }
  echo "[$spec] $(python3 -c "
import json;d=json.loads(open('$o.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('host_cpu'))")"
done
