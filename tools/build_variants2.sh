#!/usr/bin/env bash
# Like build_variants.sh, but the knobs apply to SEVERAL source files at once (FILES, default
# "mlp_f16x3 mlp_bwd": the vanilla training forward and chain):
#   tools/build_variants2.sh NAME "-DFLAG" [NAME2 "FLAGS2" ...]
set -eu
cd "$(dirname "$0")/../articulated-object-nerf_amd/csrc"
make -s -j8 ../lib/libaonerf.so
mkdir -p ../lib/variants build/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include"
FILES=${FILES:-mlp_f16x3 mlp_bwd}
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  OBJS=""
  for o in build/*.o; do
    f=$(basename "$o" .o)
    if [[ " $FILES " == *" $f "* ]]; then
      SCHED=""
      [[ "$f" == mlp_f16x3 || "$f" == mlp_art || "$f" == mlp_bwd ]] && SCHED="-mllvm -amdgpu-sched-strategy=iterative-ilp"
      /opt/rocm/bin/hipcc $FLAGS $SCHED $extra -c $f.hip -o build/variants/${f}_$name.o &
      OBJS="$OBJS build/variants/${f}_$name.o"
    else
      OBJS="$OBJS $o"
    fi
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libaonerf_$name.so $OBJS
  echo "built $name ($extra)"
done
