#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_http.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r5aw_tests.txt 2>&1 || exit 1
bash scripts/gpu_r5av.sh
