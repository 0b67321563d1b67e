#!/bin/bash
# is C3's u16 tree image (~4.07 MB at 1,000 trees) falling
# out of one XCD's 4 MB L2?  Times the first T trees of the C3 forest at 1M
# rows (us per tree per 1M rows) and, at T = 800 (image under 4 MB) and 1000
# (over), the L2 hit rate and FETCH bytes per row.  The environment passes
# through (TI_TX16=0: the record bottom's 4.07 MB image).  Usage: bash
# scripts/gpu_c3_l2.sh PREFIX [workload]
set -o pipefail
P=${1:-r5_c3_l2}; WL=${2:-c3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
for T in 250 500 700 800 900 1000; do
  timeout -k 10 120 python scripts/kernel_workload.py --workload $WL --trees $T --steps 5 >> gpurun_out/${P}.jsonl || exit 1
done
export TMPDIR=/tmp
for T in 800 1000; do
  for pass in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    n=$(echo $pass | cut -c1-5)
    (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --pmc $pass -d $ROOT/gpurun_out/${P}_T${T}_$n -o run --output-format csv -- python3 $ROOT/scripts/kernel_workload.py --workload $WL --trees $T --steps 3) > gpurun_out/${P}_T${T}_$n.log 2>&1 || exit 2
  done
done
