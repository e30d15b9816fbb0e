#!/usr/bin/env bash
# Build A/B variants of libaonerf.so that differ only in mlp_f16x3.hip compile-time knobs:
#   tools/build_variants.sh NAME "-DAON_RING=3 -DAON_CHUNK_H=32" [NAME2 "FLAGS2" ...]
# -> articulated-object-nerf_amd/lib/variants/libaonerf_NAME.so (select with AONERF_LIB=...)
set -eu
cd "$(dirname "$0")/../articulated-object-nerf_amd/csrc"
make -s -j8
mkdir -p ../lib/variants build/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include"
OTHERS=$(ls build/*.o | grep -v mlp_f16x3)
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  /opt/rocm/bin/hipcc $FLAGS -mllvm -amdgpu-sched-strategy=iterative-ilp $extra -c mlp_f16x3.hip -o build/variants/mlp_f16x3_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libaonerf_$name.so $OTHERS build/variants/mlp_f16x3_$name.o
  echo "built $name ($extra)"
done
