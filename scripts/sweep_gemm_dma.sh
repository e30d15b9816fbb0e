#!/usr/bin/env bash
set -eu
for name in default nb2 nb4 nb6; do
  if [ "$name" = default ]; then lib=articulated-object-nerf_amd/lib/libaonerf.so; else lib=articulated-object-nerf_amd/lib/variants/libaonerf_$name.so; fi
  for k in 96 128 192 256; do
    AONERF_LIB=$PWD/$lib AON_KSPLITS=$k timeout -k 10 120 python tools/prof_gemm.py 2>/dev/null
  done
done
