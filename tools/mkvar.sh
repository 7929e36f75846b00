#!/bin/bash
# A/B variant build: tools/mkvar.sh NAME 'sed expr for entropy.hip' ['sed expr for stats.hip']
# copies the sources, applies the edits and builds jpgenc_amd/lib/var/NAME/libjpge.so
# (for tools/ab_libs.sh / ab_workload.sh; nothing under var/ is a product path).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
n=$1; e=${2:-}; st=${3:-}
V=/tmp/jpge_var_$n
rm -rf $V; mkdir -p $V/jpgenc_amd; cp -r $R/jpgenc_amd/csrc $V/jpgenc_amd/; ln -s $R/include $V/include
[ -n "$e" ] && sed -i "$e" $V/jpgenc_amd/csrc/entropy.hip
[ -n "$st" ] && sed -i "$st" $V/jpgenc_amd/csrc/stats.hip
cd $R && make -s SRC=$V/jpgenc_amd/csrc BUILD=build/var_$n LIBDIR=jpgenc_amd/lib/var/$n jpgenc_amd/lib/var/$n/libjpge.so
ls -la jpgenc_amd/lib/var/$n/libjpge.so
