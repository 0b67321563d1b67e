# top depth / trees-a-lane sweeps: c3_maxbin (compact u8 bottom) and C3
# (compact u16 bottom) at 1M rows, twice
set -o pipefail
run() {  # workload variant env...
  local wl=$1 v="$2"; shift 2
  env "$@" timeout -k 10 120 python scripts/kernel_workload.py --workload $wl --steps 5 | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/r5r_sweep.jsonl || exit 2
}
for i in 1 2; do
  for ilp in 4 8; do for top in 6 7 8 9; do run c3_maxbin "ilp$ilp top$top" TI_LX_ILP=$ilp TI_TX_TOP=$top; done; done
  for cfg in "8 8" "8 9" "4 8" "4 9"; do set -- $cfg; run c3 "ilp$1 top$2" TI_TX16_ILP=$1 TI_TX_TOP=$2; done
done
