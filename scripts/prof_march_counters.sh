#!/usr/bin/env bash
# SQ counter passes over the fused coarse march alone (tools/prof_march.py), for the libraries
# named in LIBS ("default" = the in-tree build, else lib/variants/libaonerf_<name>.so).
set -u
OUT=gpurun_out/${1:-ctr_march}; shift || true
mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset AONERF_LIB; else export AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_$lib.so; fi
  timeout -k 10 120 python3 tools/prof_march.py > "$OUT/$lib.timing.json" 2>&1 || exit $?
  pass() { local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$lib/$name" -o run -- python3 tools/prof_march.py --reps 1 > "$OUT/$lib/$name.log" 2>&1
    local rc=$?; echo "$lib $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
  mkdir -p "$OUT/$lib"
  pass A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
  pass B SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM
done
echo done
