#!/bin/bash
# TreeSHAP: GPU parity tests, then the C2 contributions bench with the
# register kernel (default) and the generic kernel (TI_SHAP_GENERIC=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shap.py tests/test_gpu_tree_shard.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/shap_tests.log 2>&1
rc=$?; tail -5 gpurun_out/shap_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_configs.py --configs shap > gpurun_out/shap_reg.log 2>&1 || exit $?
tail -1 gpurun_out/shap_reg.log
TI_SHAP_GENERIC=1 timeout -k 10 300 python scripts/bench_configs.py --configs shap --rows-shap 20000 > gpurun_out/shap_gen.log 2>&1 || exit $?
tail -1 gpurun_out/shap_gen.log
exit 0
