#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes (one run each, kernel-trace only,
# no more counters per block than gfx950 allows) over one python command.
# Usage: scripts/pmc_passes.sh OUT_SUBDIR script.py [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
SCRIPT=$ROOT/$1
shift
ARGS=("$@")
run() {  # name timeout rocprof-args...
  local name=$1 to=$2; shift 2
  (cd /tmp && timeout -k 10 "$to" rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$SCRIPT" "${ARGS[@]}") > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; tail -5 "$OUT/$name.log"; exit $rc; fi
}
run stats 240 --kernel-trace --stats
run pmc_sq 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU
run pmc_ta 240 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
run pmc_tcp 240 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
run pmc_tlb 240 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run pmc_tcc 240 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
if [ -n "$PMC_HBM" ]; then
  run pmc_fetch 240 --pmc FETCH_SIZE
  run pmc_write 240 --pmc WRITE_SIZE
  run pmc_lds 240 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY
fi
exit 0
