#!/usr/bin/env bash
# Interleaved A/B of library builds on one timing tool -- the single driver for the A/B results
# in DESIGN.md (rounds 1-3 used one-off scripts per experiment; they are in git history).
#
#   scripts/ab.sh OUT TOOL [LIB...]
#
# LIB: "default" (lib/libaonerf.so) or NAME (lib/variants/libaonerf_NAME.so, built by
# tools/build_variants.sh); none given = default + every variant.  Each round runs every LIB
# once, one process each (AONERF_LIB), so box drift hits all of them alike.
# TOOL:
#   mlp        tools/prof_mlp.py --precision f16x3 --reps 4   (fused MLP alone; + --dump FILE: raw sha)
#   march      tools/prof_march.py                            (fused coarse march, median of 20)
#   composite  tools/prof_composite.py                        (per-ray kernels)
#   gemm       tools/prof_gemm.py                             (weight-gradient GEMM)
#   train      tools/prof_train_step.py                       (C5 step; --art, --precision ...)
#   bench      bench.py --no-cpu-baseline                     (every bench record)
#   bf16-sha   tools/diag/bf16_ab_outputs.py                  (sha of every bf16-step output)
#   trainrec   tools/prof_train_records.py                    (C5 records + fine-level kernel ms)
# env: ROUNDS (default 2), TOOL_ARGS (extra arguments), LIMIT (seconds per run, default 300).
# Writes OUT/NAME.ROUND.log under gpurun_out/ and prints each run's last line; stops at the
# first failing run (no retries).
set -u
OUT=gpurun_out/${1:?OUT}; TOOL=${2:?TOOL}; shift 2
case $TOOL in
  mlp) CMD="tools/prof_mlp.py --precision f16x3 --reps 4" ;;
  march) CMD="tools/prof_march.py" ;;
  composite) CMD="tools/prof_composite.py" ;;
  gemm) CMD="tools/prof_gemm.py" ;;
  train) CMD="tools/prof_train_step.py" ;;
  bench) CMD="bench.py --no-cpu-baseline" ;;
  bf16-sha) CMD="tools/diag/bf16_ab_outputs.py" ;;
  trainrec) CMD="tools/prof_train_records.py" ;;
  *) echo "unknown TOOL $TOOL"; exit 2 ;;
esac
V=articulated-object-nerf_amd/lib/variants
LIBS="$*"
if [ -z "$LIBS" ]; then
  LIBS="default"
  for so in $V/libaonerf_*.so; do [ -e "$so" ] && LIBS="$LIBS $(basename "$so" .so | sed 's/^libaonerf_//')"; done
fi
mkdir -p "$OUT"
for round in $(seq 1 "${ROUNDS:-2}"); do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset AONERF_LIB; else export AONERF_LIB=$PWD/$V/libaonerf_$lib.so; fi
    timeout -k 10 "${LIMIT:-300}" python $CMD ${TOOL_ARGS:-} > "$OUT/$lib.$round.log" 2>&1
    rc=$?
    echo "$lib round $round rc=$rc: $(grep -v amdgpu.ids "$OUT/$lib.$round.log" | tail -1 | cut -c1-300)"
    [ $rc -eq 0 ] || exit $rc
  done
done
unset AONERF_LIB
