#!/usr/bin/env bash
# Build A/B variants of libaonerf.so that differ only in some source files' compile-time knobs
# (FILE=mlp_f16x3 by default; e.g. FILE=march, or a list: FILE="mlp_f16x3 mlp_bwd"):
#   tools/build_variants.sh NAME "-DAON_RING=3 -DAON_CHUNK_H=32" [NAME2 "FLAGS2" ...]
# -> articulated-object-nerf_amd/lib/variants/libaonerf_NAME.so (select with AONERF_LIB=...)
set -eu
cd "$(dirname "$0")/../articulated-object-nerf_amd/csrc"
make -s -j8
mkdir -p ../lib/variants build/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include"
FILES=${FILE:-mlp_f16x3}
OTHERS=$(ls build/*.o)
for f in $FILES; do OTHERS=$(echo "$OTHERS" | grep -v "/$f.o"); done
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  VOBJS=""
  for f in $FILES; do
    SCHED=""  # the Makefile's per-file scheduler choice
    case $f in mlp_f16x3|mlp_art|mlp_bwd) SCHED="-mllvm -amdgpu-sched-strategy=iterative-ilp" ;; esac
    /opt/rocm/bin/hipcc $FLAGS $SCHED $extra -c $f.hip -o build/variants/${f}_$name.o
    VOBJS="$VOBJS build/variants/${f}_$name.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libaonerf_$name.so $OTHERS $VOBJS
  echo "built $name ($extra)"
done
