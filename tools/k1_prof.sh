#!/bin/bash
# Kernel-trace durations of K1 micro-bench binaries (diagnostic): tools/k1_prof.sh name...
set -u
export TMPDIR=/tmp
for n in "$@"; do
  d=gpurun_out/k1prof_$n
  rm -rf "$d"; mkdir -p "$d"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- build/k1/k1_$n 3840 2160 16 10 90 > "$d/log" 2>&1 || { echo "$n failed"; tail -5 "$d/log"; exit 1; }
  f=$(find "$d" -name '*kernel_stats.csv' | head -1)
  echo "== $n: $(grep -h 'K1 ' "$d/log")"
  grep fdct "$f" | awk -F, '{printf "   calls %s  avg %.2f us  min %.2f us  max %.2f us\n", $3, $5/1000, $6/1000, $7/1000}'
done
