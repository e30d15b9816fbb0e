#!/usr/bin/env bash
# Round-4 late session: C5 step timings after the batching change, the non-temporal kept-store
# A/B (lib/variants/libaonerf_nt.so), then the training GPU tests the changes touch.
set -u
OUT=gpurun_out/r04_late; mkdir -p $OUT
for a in "--precision bf16" "--precision bf16 --art" "--precision f16x3 --art" "--precision f16x3"; do
  timeout -k 10 120 python3 tools/prof_train_step.py --steps 20 $a || exit 1
done
ROUNDS=2 TOOL_ARGS="--steps 20 --precision bf16" bash scripts/ab.sh r04_late/ab_nt_bf16 train default nt || exit 1
ROUNDS=2 TOOL_ARGS="--steps 10 --precision bf16 --art" bash scripts/ab.sh r04_late/ab_nt_artbf16 train default nt || exit 1
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_train_bf16.py tests/test_gpu_art_train_bf16.py tests/test_gpu_art_train.py -k "not trajectory" \
  > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
