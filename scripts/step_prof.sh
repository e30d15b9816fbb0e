#!/usr/bin/env bash
# Kernel traces of the C5 training steps (tools/prof_train_step.py) and their last-step breakdown
# (scripts/step_breakdown.py).  Usage on the box: bash scripts/step_prof.sh OUTDIR [modes...]
# modes: art_bf16 bf16 art f16x3 (default: art_bf16 bf16)
set -u
OUT=${1:-gpurun_out/step}; shift || true
MODES=${*:-art_bf16 bf16}
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in $MODES; do
  case $m in
    art_bf16) a="--art --precision bf16" ;;
    art_bf16_view) a="--art --precision bf16 --view" ;;
    art_bf16_f16w) a="--art --precision bf16 --f16w 1" ;;
    art_bf16_f16x) a="--art --precision bf16 --f16w 0 --f16x 1" ;;
    art_bf16_f16x3) a="--art --precision bf16 --f16w 0 --f16x 0" ;;
    art) a="--art --precision f16x3" ;;
    bf16) a="--precision bf16" ;;
    f16x3) a="--precision f16x3" ;;
  esac
  echo "== $m"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$m" -o run -- \
    python3 tools/prof_train_step.py $a --steps 8 > "$OUT/$m.log" 2>&1
  rc=$?
  echo "== $m rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  f=$(find "$OUT/$m" -name '*kernel_trace.csv' | head -1)
  python3 scripts/step_breakdown.py "$f" > "$OUT/$m.txt" && head -1 "$OUT/$m.txt"
done
