set -u
OUT=gpurun_out/train_ab; mkdir -p $OUT
export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_base.so; else unset AONERF_LIB; fi
  timeout -k 10 300 python tools/bench_train.py > $OUT/$v.log 2>&1 || exit 3
  echo "$v: $(tail -1 $OUT/$v.log | cut -c1-400)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > $OUT/kt_$v.log 2>&1 || exit 4
done
