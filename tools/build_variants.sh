#!/usr/bin/env bash
# Build A/B variants of libaonerf.so that differ only in one source file's compile-time knobs
# (FILE=mlp_f16x3 by default; e.g. FILE=march):
#   tools/build_variants.sh NAME "-DAON_RING=3 -DAON_CHUNK_H=32" [NAME2 "FLAGS2" ...]
# -> articulated-object-nerf_amd/lib/variants/libaonerf_NAME.so (select with AONERF_LIB=...)
set -eu
cd "$(dirname "$0")/../articulated-object-nerf_amd/csrc"
make -s -j8
mkdir -p ../lib/variants build/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include"
FILE=${FILE:-mlp_f16x3}
SCHED=""
[ "$FILE" = mlp_f16x3 ] && SCHED="-mllvm -amdgpu-sched-strategy=iterative-ilp"
OTHERS=$(ls build/*.o | grep -v "/$FILE.o")
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  /opt/rocm/bin/hipcc $FLAGS $SCHED $extra -c $FILE.hip -o build/variants/${FILE}_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libaonerf_$name.so $OTHERS build/variants/${FILE}_$name.o
  echo "built $name ($extra)"
done
