#!/usr/bin/env bash
# SQ / TCC counter passes over one launch of the f16_single weight-gradient batch
# (tools/prof_f1.py), one pass per group; summary by scripts/ctr_summary.py.
set -u
OUT=gpurun_out/${1:-ctr_f1}; shift || true
mkdir -p "$OUT"; export TMPDIR=/tmp
pass() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_f1.py > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python3 tools/prof_f1.py --reps 5 > "$OUT/timing.log" 2>&1 || exit $?
pass A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
pass C TCC_HIT_sum TCC_MISS_sum GRBM_COUNT
python3 scripts/ctr_summary.py "$OUT" "$OUT/summary.json" k_gemm_f1_256_batch > "$OUT/summary.log" 2>&1
cat "$OUT/timing.log" "$OUT/summary.log"
