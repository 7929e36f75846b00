#!/bin/bash
# Build libjpge from a git revision (default HEAD) as variant "head" (or $2) for
# A/B runs against the working tree: jpgenc_amd/lib/var/<name>/libjpge.so
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
rev=${1:-HEAD}; name=${2:-head}
wt=$R/build/wt_$name
rm -rf "$wt"; git -C "$R" worktree prune
git -C "$R" worktree add -f --detach "$wt" "$rev" > /dev/null
make -s -C "$wt" -j8 jpgenc_amd/lib/libjpge.so
mkdir -p "$R/jpgenc_amd/lib/var/$name"
cp "$wt/jpgenc_amd/lib/libjpge.so" "$R/jpgenc_amd/lib/var/$name/libjpge.so"
git -C "$R" worktree remove --force "$wt"
