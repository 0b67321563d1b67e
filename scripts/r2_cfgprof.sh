#!/bin/bash
# PMC passes for the C3 / C4 kernels at 1M rows (bench.py's c3/c4 roofline keys)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
prof() {  # out config settings
  local OUT=$ROOT/gpurun_out/$1 CFG=$2 SET=$3
  mkdir -p "$OUT"
  run() {
    local name=$1; shift
    (cd /tmp && timeout -k 10 120 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/scripts/explicit_sweep.py" --configs "$CFG" --steps 2 --settings "$SET") > "$OUT/$name.log" 2>&1
    local rc=$?; echo "rc=$rc $name" | tee -a "$OUT/steps.log"; return $rc
  }
  run stats --kernel-trace --stats || return 1
  run pmc_a --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD || return 1
  run pmc_b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE || return 1
  run pmc_t --pmc TA_BUSY_avr TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || return 1
  run pmc_c --pmc TCC_HIT_sum TCC_MISS_sum || return 1
  run pmc_f --pmc FETCH_SIZE || return 1
  run pmc_w --pmc WRITE_SIZE || return 1
}
# usage: scripts/r2_cfgprof.sh [OUTNAME CONFIG SETTING]...  (default: C3 layout 7, C4 layout 8)
if [ $# -eq 0 ]; then set -- r2_c3_l7c c3 lexplicit:7 r2_c4_l8 c4 hexplicit:8; fi
while [ $# -ge 3 ]; do
  prof "$1" "$2" "$3" || exit 1
  shift 3
done
