#!/usr/bin/env bash
# PMC passes over tools/prof_gemm.py (the fine-level dW GEMMs): latency, TLB, wave waits.
set -u
OUT=gpurun_out/${1:-pmc_gemm2}; mkdir -p "$OUT"; export TMPDIR=/tmp
pass() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_gemm.py > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass lat TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
pass tcc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_TAG_STALL_sum
echo done
