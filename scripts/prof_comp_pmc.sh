#!/usr/bin/env bash
# Instruction mix of the per-ray kernels (tools/prof_composite.py) from SQ counters.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/comp_pmc; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o run -- python3 tools/prof_composite.py --reps 2 > $OUT/p1.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 tools/prof_composite.py --reps 2 > $OUT/p2.log 2>&1 || exit 4
echo ok
