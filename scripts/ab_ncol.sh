#!/usr/bin/env bash
# Time lib variants x {NCOL=1, NCOL=2} on the MLP alone (interleaved rounds, one process each).
set -u
OUT=gpurun_out/${1:-abn}; mkdir -p "$OUT"
for round in 1 2; do
  for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
    for nc in ${NCOLS:-1 2}; do
      name=$(basename "$so" .so)_nc$nc
      AON_F16X3_NCOL=$nc AONERF_LIB=$so timeout -k 10 120 python tools/prof_mlp.py --precision f16x3 --reps 4 > "$OUT/$name.$round.log" 2>&1
      rc=$?; echo "$name round $round rc=$rc: $(grep f16x3 "$OUT/$name.$round.log" | tail -1)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
