#!/usr/bin/env bash
# GPU-box session for the training path: training tests, training bench, kernel trace.
# Usage: bash scripts/train_round.sh [tag] [bench_train args...]
set -u
TAG=${1:-tr01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_train 600 python -m pytest tests/test_gpu_train.py -m gpu -q -s -p no:cacheprovider
step bench_train 600 python tools/bench_train.py "$@"
tail -1 "$OUT/bench_train.log" > "$OUT/bench_train.json"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
step rocprof_train 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 "$@"
echo done
