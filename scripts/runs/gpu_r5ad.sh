# round 5: the serving GPU tests after the sklearn / lgbserver native routes
set -o pipefail
mkdir -p gpurun_out/r5ad
timeout -k 10 400 python -u -m pytest tests/test_gpu_native_http.py tests/test_gpu_native_batcher.py tests/test_gpu_server.py tests/test_gpu_c5_serving.py tests/test_gpu_v2.py -v --timeout 150 --timeout-method thread > gpurun_out/r5ad/serving_tests.txt 2>&1 || exit 1
