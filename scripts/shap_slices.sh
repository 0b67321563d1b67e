#!/bin/bash
# TreeSHAP path slices: GPU parity tests, then the C2 contributions bench at
# 100k and 4k rows with the default path math and with float64 path math forced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shap.py tests/test_gpu_tree_shard.py -m gpu -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/shap_tests.log 2>&1
rc=$?; tail -15 gpurun_out/shap_tests.log; [ $rc -gt 1 ] && exit $rc
for rows in 100000 4096; do
  timeout -k 10 300 python scripts/bench_configs.py --configs shap --rows-shap $rows > gpurun_out/shap_auto_$rows.log 2>&1 || exit $?
  tail -1 gpurun_out/shap_auto_$rows.log
  TI_SHAP_F64=1 timeout -k 10 300 python scripts/bench_configs.py --configs shap --rows-shap $rows > gpurun_out/shap_f64_$rows.log 2>&1 || exit $?
  tail -1 gpurun_out/shap_f64_$rows.log
done
exit 0
