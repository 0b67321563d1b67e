#!/bin/bash
# Parity subset of the explicit/record layouts, then an A/B of variant
# libraries on C3/C4: scripts/ab_check.sh "c3,c4" default name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4_full.py -k "every_layout or zero_missing or record_layouts or leafwise or c4" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/sweep_configs.sh "$@"
