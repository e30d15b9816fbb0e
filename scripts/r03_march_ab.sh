mkdir -p gpurun_out/r03f
timeout -k 10 120 python tools/diag/march_dbg.py > gpurun_out/r03f/dbg.log 2>&1; echo dbg_rc=$?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "march" -v --timeout 200 --timeout-method thread -s -p no:cacheprovider > gpurun_out/r03f/pytest_march.log 2>&1; echo march_rc=$?
V=articulated-object-nerf_amd/lib/variants
for i in 1 2; do
  for lib in default v1 occ6 rows0; do
    if [ $lib = default ]; then L=""; else L=$V/libaonerf_$lib.so; fi
    env ${L:+AONERF_LIB=$L} timeout -k 10 120 python tools/prof_composite.py >> gpurun_out/r03f/prof_$lib.json 2>&1 || echo fail_$lib
  done
done
echo prof_done
