#!/bin/bash
# TreeSHAP path-slice sweep on the C2 model (100k rows): automatic, then forced slice counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in 0 5 20 40; do
  TI_SHAP_SLICES=$s timeout -k 10 300 python scripts/bench_configs.py --configs shap --rows-shap 100000 > gpurun_out/sweep_s$s.log 2>&1 || exit $?
  echo "slices=$s $(grep -o '"rows_per_s": [0-9.e+]*' gpurun_out/sweep_s$s.log | head -1)"
done
exit 0
