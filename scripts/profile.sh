#!/bin/bash
# rocprofv3 evidence for the C2 bench kernel: kernel-trace stats + PMC passes
# (each --pmc pass is its own run, kernel-trace only, per the pool's rules).
# Usage: scripts/profile.sh [out-subdir]   (kernel env knobs pass through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  (cd /tmp && timeout -k 10 "$to" rocprofv3 "$@" -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --latency-qps 0 --nan-variant 0) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
run stats 300 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv
run pmc_a 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_a" -o run --output-format csv
run pmc_b 300 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d "$OUT/pmc_b" -o run --output-format csv
run pmc_c 300 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL -d "$OUT/pmc_c" -o run --output-format csv
run pmc_d 300 --pmc FETCH_SIZE -d "$OUT/pmc_d" -o run --output-format csv
run pmc_e 300 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_e" -o run --output-format csv
exit 0
