#!/bin/bash
# PMC passes (LDS-side counters) for the staged record kernel on C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
prof() {  # out settings
  local OUT=$ROOT/gpurun_out/$1 SET=$2
  mkdir -p "$OUT"
  run() {
    local name=$1; shift
    (cd /tmp && timeout -k 10 120 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/scripts/explicit_sweep.py" --configs c3 --steps 2 --settings "$SET") > "$OUT/$name.log" 2>&1
    local rc=$?; echo "rc=$rc $name" | tee -a "$OUT/steps.log"; return $rc
  }
  run stats --kernel-trace --stats || return 1
  run pmc_a --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES || return 1
  run pmc_b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_MEM_VIOLATIONS SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE || return 1
  run pmc_c --pmc SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM || return 1
}
prof r2_c3_l7b lexplicit:7 || exit 1

