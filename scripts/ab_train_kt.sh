#!/usr/bin/env bash
# Training A/B (scripts/ab_train_variants.sh) + per-kernel times of each variant + all GPU tests.
set -u
export TMPDIR=/tmp
bash scripts/ab_train_variants.sh train_kt || exit $?
OUT=gpurun_out/train_kt
for so in articulated-object-nerf_amd/lib/variants/libaonerf_*.so; do
  v=$(basename $so .so)
  AONERF_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > $OUT/kt_$v.log 2>&1 || exit 4
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; echo "gpu tests rc=$?"; tail -1 $OUT/pytest_gpu.log
