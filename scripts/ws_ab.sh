#!/usr/bin/env bash
# A/B of the render MLP dataflows on one box: for each weight-streamed configuration
# (AON_WS_WAVES / AON_WS_PIPE), the bit-equality tests against the LDS-ring kernel and the
# interleaved timing of both on the bench frame's fine level (tools/prof_mlp_ws.py), vanilla and
# articulated.  Usage: bash scripts/ws_ab.sh OUT "8:0 4:0 8:1" (waves:pipe pairs)
set -u
OUT=gpurun_out/${1:?OUT}; CONFIGS=${2:-"8:0 4:0 8:1"}
mkdir -p "$OUT"; export TMPDIR=/tmp
for cfg in $CONFIGS; do
  wv=${cfg%%:*}; pp=${cfg##*:}
  export AON_WS_WAVES=$wv AON_WS_PIPE=$pp
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_articulated.py -k ws_equals_streamed > "$OUT/test_$wv$pp.log" 2>&1 || { echo "test $cfg failed"; tail -5 "$OUT/test_$wv$pp.log"; exit 1; }
  timeout -k 10 200 python -u tools/prof_mlp_ws.py > "$OUT/prof_$wv$pp.log" 2>&1 || exit 1
  timeout -k 10 200 python -u tools/prof_mlp_ws.py --art --rays 76800 > "$OUT/prof_art_$wv$pp.log" 2>&1 || exit 1
  echo "$cfg: $(tail -1 "$OUT/test_$wv$pp.log")"
  echo "  vanilla $(tail -1 "$OUT/prof_$wv$pp.log")"
  echo "  art     $(tail -1 "$OUT/prof_art_$wv$pp.log")"
done
