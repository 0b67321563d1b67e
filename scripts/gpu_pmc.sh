# PMC passes of the bench kernels (scripts/kernel_pmc.sh per workload) and
# their condensed per-launch figures (scripts/make_pmc_json.py), for bench.py's
# rooflines.  Usage: bash scripts/gpu_pmc.sh PREFIX workload...
set -o pipefail
P=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in "$@"; do
  case $w in
    c2|c2_hist) k=bheap_fix_kernel; lay=bheap; extra="--walk-id 2 --walk-step fixed-layout-walk,scalar-root --model-bytes 2800000" ;;
    c3|c3_f64) k=t16split_predict_kernel; lay=texplicit; extra="" ;;
    c3_maxbin) k=t8explicit_predict_kernel; lay=texplicit; extra="" ;;
    c4) k=hexplicit_predict_kernel; lay=hexplicit; extra="" ;;
  esac
  xb=1; [ "$w" = c2 ] && xb=3
  bash scripts/kernel_pmc.sh ${P}_$w $w --steps 3 --x-buffers $xb || exit 1
  python scripts/make_pmc_json.py gpurun_out/${P}_$w "$k" $w $lay 1000000 gpurun_out/${P}_${w}_pmc.json \
      --source "profiles/${P}_${w}_* (scripts/kernel_pmc.sh ${P}_$w $w)" $extra > /dev/null || exit 2
done
