#!/bin/bash
# C4 against one XCD's 4 MB L2: the first T trees (and 25-tree slices from the
# middle and end) of the 200-tree, ~30 MB C4 forest at 1M rows; per-tree cost
# and, at T = 25 and 200, the L2 hit rate / FETCH bytes.  Decides whether
# tree passes sized to one XCD's L2 pay.
set -o pipefail
P=${1:-r6m_c4_slices}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out
for spec in "25 0" "50 0" "100 0" "200 0" "25 100" "25 175" "12 0" "12 188"; do
  set -- $spec
  timeout -k 10 150 python scripts/kernel_workload.py --workload c4 --trees $1 --tree-start $2 --steps 5 >> gpurun_out/${P}.jsonl || exit 1
done
export TMPDIR=/tmp
for T in 25 200; do
  for pass in "TCC_HIT_sum TCC_MISS_sum TD_TD_BUSY_sum TD_TC_STALL_sum" "FETCH_SIZE"; do
    n=$(echo $pass | cut -c1-5)
    (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --pmc $pass -d $ROOT/gpurun_out/${P}_T${T}_$n -o run --output-format csv -- python3 $ROOT/scripts/kernel_workload.py --workload c4 --trees $T --steps 3) > gpurun_out/${P}_T${T}_$n.log 2>&1 || exit 2
  done
done
