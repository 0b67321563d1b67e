#!/bin/bash
# Round 5: compact u16 bottom on one workload at 1M rows -- trees per lane
# (TI_TX16_ILP) and top depth (TI_TX_TOP, 0 = no heap top), beside the record
# bottom (TI_TX16=0), twice.  Usage: bash scripts/gpu_t16_sweep.sh PREFIX WORKLOAD
set -o pipefail
P=${1:-r5e}; WL=${2:-c3}
mkdir -p gpurun_out
run() {  # variant env...
  local v="$1"; shift
  env "$@" timeout -k 10 120 python scripts/kernel_workload.py --workload $WL --steps 5 | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/${P}_sweep.jsonl || exit 2
}
for i in 1 2; do
  run "records" TI_TX16=0
  for ilp in 8 12 16; do
    for top in 0 6 7 8; do
      run "ilp$ilp top$top" TI_TX16_ILP=$ilp TI_TX_TOP=$top
    done
  done
done
