#!/bin/bash
# TreeSHAP slice sweep, packed build: 100k rows (auto = 42 slices, 64) and 1M rows (auto = 4 slices, 16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "100000 0" "100000 64" "1000000 0" "1000000 16"; do
  set -- $cfg
  TI_SHAP_SLICES=$2 timeout -k 10 300 python scripts/bench_configs.py --configs shap --rows-shap $1 > gpurun_out/sw_$1_$2.log 2>&1 || exit $?
  echo "rows=$1 slices=$2 $(grep -o '"rows_per_s": [0-9.e+]*' gpurun_out/sw_$1_$2.log | head -1)"
done
exit 0
