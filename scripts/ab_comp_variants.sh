#!/usr/bin/env bash
# Interleaved timing of every lib/variants/libaonerf_*.so on the per-ray kernels (tools/prof_composite.py).
set -u
OUT=gpurun_out/${1:-comp_var}; mkdir -p $OUT
for r in 1 2 3; do for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
  v=$(basename $so .so)
  AONERF_LIB=$so timeout -k 10 120 python tools/prof_composite.py > $OUT/$v.$r.json 2>$OUT/$v.$r.err || exit 3
  echo "$v $r: $(cat $OUT/$v.$r.json)"
done; done
