#!/usr/bin/env bash
# March kernel A/B session: bit-exactness tests, then interleaved timing of the in-tree build and
# the variants named in LIBS (tools/prof_march.py, median of 20 launches, 3 rounds).
set -u
OUT=gpurun_out/${1:-march_ab}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "march" -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_march.log" 2>&1
echo "march tests rc=$?"
V=articulated-object-nerf_amd/lib/variants
for i in 1 2 3; do
  for lib in default ${LIBS:-}; do
    if [ "$lib" = default ]; then unset AONERF_LIB; else export AONERF_LIB=$V/libaonerf_$lib.so; fi
    timeout -k 10 120 python tools/prof_march.py | grep '^{' >> "$OUT/$lib.jsonl" || { echo "fail $lib"; exit 1; }
  done
done
unset AONERF_LIB
for f in "$OUT"/*.jsonl; do echo "$f $(python3 -c "import json,sys; print(sorted(round(json.loads(l)['ms'],4) for l in open('$f')))")"; done
