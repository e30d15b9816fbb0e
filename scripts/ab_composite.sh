set -u
OUT=gpurun_out/comp_ab; mkdir -p $OUT
for r in 1 2; do for v in base new; do
  AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_$v.so timeout -k 10 120 python tools/prof_composite.py > $OUT/$v.$r.json 2>$OUT/$v.$r.err || exit 3
  echo "$v $r: $(cat $OUT/$v.$r.json)"
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 $OUT/pytest_gpu.log
