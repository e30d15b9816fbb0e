#!/usr/bin/env bash
# Time every lib/variants/libaonerf_*.so on the training steps (vanilla + articulated),
# interleaved rounds, one process each:  bash scripts/ab_train.sh [tag]
set -u
OUT=gpurun_out/${1:-ab_train}; mkdir -p "$OUT"
for round in 1 2; do
  for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
    name=$(basename "$so" .so)
    for model in vanilla art; do
      AONERF_LIB=$so timeout -k 10 200 python tools/bench_train.py --model $model > "$OUT/$name.$model.$round.log" 2>&1
      rc=$?; echo "$name $model round $round rc=$rc: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.$model.$round.log")"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
