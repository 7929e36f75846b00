#!/bin/bash
# K1 micro A/B (diagnostic): each binary in jpgenc_amd/bin/k1/ alternately, 3 rounds.
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/k1ab
for r in 1 2 3; do
  for b in "$@"; do
    timeout -k 10 60 ./jpgenc_amd/bin/k1/k1_$b 3840 2160 16 20 90 > gpurun_out/k1ab/$b.$r.txt 2>&1 || exit 1
    echo "$b: $(grep kernel-exact gpurun_out/k1ab/$b.$r.txt)"
  done
done
[ -x jpgenc_amd/bin/k1/k1_stamps ] && timeout -k 10 60 ./jpgenc_amd/bin/k1/k1_stamps 3840 2160 16 5 90
true
