#!/usr/bin/env bash
# A/B of a library build on one C5 training step: kernel traces of tools/prof_train_step.py with
# the release library and with AONERF_LIB=<alt>, alternated twice, and their breakdowns.
# Usage on the box: bash scripts/ab_lib_step.sh OUTDIR ALT_SO "<prof_train_step args>"
set -u
OUT=$1; ALT=$2; ARGS=$3
mkdir -p "$OUT"
export TMPDIR=/tmp
for run in rel1 alt1 rel2 alt2; do
  case $run in
    rel*) lib=$PWD/articulated-object-nerf_amd/lib/libaonerf.so ;;
    alt*) lib=$PWD/$ALT ;;
  esac
  AONERF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$run" -o run -- \
    python3 tools/prof_train_step.py $ARGS --steps 8 > "$OUT/$run.log" 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "$run rc=$rc"; exit $rc; }
  f=$(find "$OUT/$run" -name '*kernel_trace.csv' | head -1)
  python3 scripts/step_breakdown.py "$f" > "$OUT/$run.txt" && echo "$run $(tail -1 "$OUT/$run.txt")"
done
