#!/usr/bin/env bash
# A/B of MLP library variants (tools/build_variants.sh): timing (interleaved rounds) + bit-identity
# of the raw outputs against the first variant.
set -u
OUT=gpurun_out/${1:-ab_persist}; mkdir -p "$OUT"
rm -f "$OUT/sha.txt"
for round in 1 2; do
  for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
    name=$(basename "$so" .so)
    AONERF_LIB=$so timeout -k 10 120 python tools/prof_mlp.py --precision f16x3 --reps 4 --dump "$OUT/sha.txt" > "$OUT/$name.$round.log" 2>&1
    rc=$?; echo "$name round $round rc=$rc: $(grep f16x3 "$OUT/$name.$round.log" | tail -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
cat "$OUT/sha.txt"
