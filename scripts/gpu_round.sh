#!/usr/bin/env bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + HBM counters.
# Usage (from the repo root, on the box):  bash scripts/gpu_round.sh [tag] [bench args...]
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: run, log, stop the session on crash/timeout
  local name=$1 lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 1100 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread
step bench 600 python bench.py "$@"
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
if [ "${EXTRA:-0}" = 1 ]; then
  step bench_art 600 python tools/bench_articulated.py
  tail -1 "$OUT/bench_art.log" > "$OUT/bench_art.json"
  step bench_train 600 python tools/bench_train.py
  tail -1 "$OUT/bench_train.log" > "$OUT/bench_train.json"
fi
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
step rocprof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@"
if [ "${EXTRA:-0}" = 1 ]; then
  step rocprof_kt_art 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_art" -o run -- python3 tools/bench_articulated.py --steps 3 --warmup 1
fi
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
step rocprof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@"
# effective clock under load (MI355X_MICROARCH.md 'DVFS give-back': GRBM_GUI_ACTIVE / 8 / wall)
step rocprof_clock 600 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_clock" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@"
step rocprof_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@"
echo done
