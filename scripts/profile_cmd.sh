#!/bin/bash
# rocprofv3 kernel-trace stats + the PMC passes of profile.sh for any python
# command.  Usage: scripts/profile_cmd.sh OUT_SUBDIR script.py [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
SCRIPT=$ROOT/$1
shift
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  (cd /tmp && timeout -k 10 "$to" rocprofv3 "$@" -- python3 "$SCRIPT" "${ARGS[@]}") > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
ARGS=("$@")
run stats 300 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv
run pmc_a 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_a" -o run --output-format csv
run pmc_b 300 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d "$OUT/pmc_b" -o run --output-format csv
run pmc_c 300 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d "$OUT/pmc_c" -o run --output-format csv
run pmc_d 300 --pmc FETCH_SIZE -d "$OUT/pmc_d" -o run --output-format csv
run pmc_e 300 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_e" -o run --output-format csv
exit 0
