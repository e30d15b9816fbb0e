#!/usr/bin/env bash
# Training-step A/B of lib/variants/libaonerf_*.so (tools/bench_train.py, interleaved rounds),
# then the GPU training tests on the default library.
set -u
OUT=gpurun_out/${1:-train_var}; mkdir -p $OUT
for r in 1 2; do for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
  v=$(basename $so .so)
  AONERF_LIB=$so timeout -k 10 300 python tools/bench_train.py > $OUT/$v.$r.log 2>&1 || exit 3
  echo "$v $r: $(tail -1 $OUT/$v.$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), "ms/step")')"
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_art_train.py -x -q --timeout 300 -p no:cacheprovider > $OUT/pytest_train.log 2>&1; echo "train tests rc=$?"; tail -2 $OUT/pytest_train.log
