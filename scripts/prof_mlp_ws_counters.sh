#!/usr/bin/env bash
# SQ / TCC counter passes over the render MLP's two dataflows (tools/prof_mlp_ws.py: interleaved
# k_mlp_fwd_f16x3 and k_mlp_ws_f16x3 launches on the bench frame's fine level); one rocprofv3
# --pmc pass per group; summary: python scripts/train_ctr_summary.py gpurun_out/OUT.
#   scripts/prof_mlp_ws_counters.sh r04f [--art]
set -u
OUT=gpurun_out/${1:-mlpws}; shift || true
mkdir -p "$OUT"; export TMPDIR=/tmp
pass() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_mlp_ws.py --reps 2 --rays 76800 ${PROF_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
pass C FETCH_SIZE
pass D WRITE_SIZE
echo done
