#!/usr/bin/env bash
# SQ / TCC counter passes over the MLP kernel alone (tools/prof_mlp.py); one pass per group.
set -u
OUT=gpurun_out/${1:-ctr}; shift || true
mkdir -p "$OUT"; export TMPDIR=/tmp
pass() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_mlp.py --reps 1 ${PROF_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python3 tools/prof_mlp.py ${PROF_ARGS:-} > "$OUT/timing.log" 2>&1 || exit $?
want() { case " ${PASSES:-A B C} " in *" $1 "*) return 0;; esac; return 1; }
want A && pass A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
want B && pass B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
want C && pass C TCC_HIT_sum TCC_MISS_sum GRBM_COUNT
want D && pass D SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
echo done
