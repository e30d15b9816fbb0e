#!/usr/bin/env bash
# SQ counter passes over the training step's fused kernels (tools/prof_train_step.py, 2 steps);
# one rocprofv3 --pmc pass per group; summary: scripts/train_ctr_summary.py OUT.
#   PROF_ARGS="--precision bf16" scripts/prof_train_counters.sh r03q
set -u
OUT=gpurun_out/${1:-trctr}; shift || true
mkdir -p "$OUT"; export TMPDIR=/tmp
pass() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_train_step.py --steps 2 ${PROF_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
# memory passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes; FETCH doubled
# on gfx950 in the summary) and the wait / store-issue mix
pass C FETCH_SIZE
pass D WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 tools/prof_train_step.py --steps 2 ${PROF_ARGS:-} > "$OUT/kt.log" 2>&1
echo "kt rc=$?"
pass E SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM_WR SQ_WAVE_CYCLES
echo done
