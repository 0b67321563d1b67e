#!/bin/bash
# rocprofv3 passes over one workload of scripts/kernel_workload.py: kernel
# stats, then one run per PMC pass (counters within gfx950's per-block slots:
# MI355X_MICROARCH.md "rocprofv3 PMC slots"), each with --kernel-trace so the
# pass's own kernel durations sit beside its counters (the passes that carry
# GRBM_GUI_ACTIVE give the profiled run's clock).  No pass combines --pmc
# with a runtime/sys trace.  Condense with scripts/make_pmc_json.py.
# Usage: scripts/kernel_pmc.sh OUT_SUBDIR WORKLOAD [kernel_workload.py args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
WL=$2
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
# A/B knobs passed in the environment (TI_TX16=0 ...) need the developer gate
export TI_DEV_KNOBS=${TI_DEV_KNOBS:-1}
run() {  # name rocprof-args...
  local name=$1; shift
  (cd /tmp && timeout -k 10 150 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/scripts/kernel_workload.py" --workload "$WL" "${ARGS[@]}") > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; tail -5 "$OUT/$name.log"; exit $rc; fi
}
ARGS=("$@")
run stats --kernel-trace --stats
run pmc_a --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run pmc_b --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
run pmc_t --kernel-trace --pmc TA_BUSY_avr TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
run pmc_c --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_f --kernel-trace --pmc FETCH_SIZE
run pmc_w --kernel-trace --pmc WRITE_SIZE
exit 0
