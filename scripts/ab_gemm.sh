#!/usr/bin/env bash
# A/B of weight-gradient GEMM builds (tools/prof_gemm.py): scripts/ab_gemm.sh OUTDIR NAME...
# (NAME "default" = lib/libaonerf.so, else lib/variants/libaonerf_NAME.so), 2 interleaved rounds
set -eu
out=$1; shift
mkdir -p "$out"
for round in 1 2; do
  for name in "$@"; do
    if [ "$name" = default ]; then lib=articulated-object-nerf_amd/lib/libaonerf.so
    else lib=articulated-object-nerf_amd/lib/variants/libaonerf_$name.so; fi
    AONERF_LIB=$PWD/$lib timeout -k 10 120 python tools/prof_gemm.py | tee "$out/$name.$round.json"
  done
done
