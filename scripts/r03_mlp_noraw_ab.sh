#!/usr/bin/env bash
# Fused-pipeline question: the fine-level MLP launch with and without its raw store
# (timing-only variant lib/variants/libaonerf_noraw.so), interleaved, 3 rounds.
set -u
OUT=gpurun_out/${1:-mlp_noraw}; mkdir -p "$OUT"
V=articulated-object-nerf_amd/lib/variants
for i in 1 2 3; do
  for lib in default noraw; do
    if [ "$lib" = default ]; then unset AONERF_LIB; else export AONERF_LIB=$V/libaonerf_$lib.so; fi
    timeout -k 10 180 python tools/prof_mlp.py --precision f16x3 --rays 307200 --reps 5 | grep f16x3 >> "$OUT/$lib.txt" || { echo "fail $lib"; exit 1; }
  done
done
unset AONERF_LIB
tail -n 15 "$OUT"/*.txt
