#!/usr/bin/env bash
# bf16 step A/B: sha of every output + step times, pre-change library vs the current one
# (tools/diag/bf16_ab_outputs.py), then the bf16 GPU tests on the current library.
set -eu
mkdir -p gpurun_out/r03o
AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_preB.so timeout -k 10 300 python -u tools/diag/bf16_ab_outputs.py 2>/dev/null | grep '^{' > gpurun_out/r03o/ab_pre.json
timeout -k 10 300 python -u tools/diag/bf16_ab_outputs.py 2>/dev/null | grep '^{' > gpurun_out/r03o/ab_new.json
AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_preB.so timeout -k 10 300 python -u tools/diag/bf16_ab_outputs.py 2>/dev/null | grep '^{' > gpurun_out/r03o/ab_pre2.json
python - <<'PY'
import json
a = json.load(open("gpurun_out/r03o/ab_pre.json")); b = json.load(open("gpurun_out/r03o/ab_new.json"))
a2 = json.load(open("gpurun_out/r03o/ab_pre2.json"))
for k in a:
    if isinstance(a[k], dict):
        diff = [n for n in a[k] if a[k][n] != b[k][n]]
        print(k, "identical" if not diff else f"{len(diff)} differ: {diff[:6]}")
    elif k.endswith("_ms"):
        print(k, f"pre {a[k]:.3f} / {a2[k]:.3f}  new {b[k]:.3f}")
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_bf16.py tests/test_gpu_art_train_bf16.py > gpurun_out/r03o/pytest_bf16.log 2>&1
tail -2 gpurun_out/r03o/pytest_bf16.log
