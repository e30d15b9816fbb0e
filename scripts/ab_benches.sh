#!/usr/bin/env bash
# End-to-end A/B of lib/variants/libaonerf_*.so: render, articulated render and training benches
# (interleaved rounds), then the GPU tests on the default library.
set -u
OUT=gpurun_out/${1:-ab_benches}; mkdir -p $OUT
for r in 1 2; do for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
  v=$(basename $so .so)
  for b in "bench.py --no-cpu-baseline" "tools/bench_articulated.py" "tools/bench_train.py" "tools/bench_train.py --model art"; do
    AONERF_LIB=$so timeout -k 10 300 python $b > $OUT/tmp.log 2>&1 || exit 3
    echo "$v $r [$b]: $(tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],2), "ms")')"
  done
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; echo "gpu tests rc=$?"; tail -1 $OUT/pytest_gpu.log
