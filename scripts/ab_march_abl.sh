#!/usr/bin/env bash
# march ablations (timing only): tools/prof_composite.py per library, 2 rounds
set -eu
for r in 1 2; do for name in default nopdf nocomp; do
  if [ "$name" = default ]; then lib=articulated-object-nerf_amd/lib/libaonerf.so; else lib=articulated-object-nerf_amd/lib/variants/libaonerf_$name.so; fi
  AONERF_LIB=$PWD/$lib timeout -k 10 120 python tools/prof_composite.py 2>/dev/null | tail -1
done; done
