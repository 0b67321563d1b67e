# round 5: the native HTTP front end on the GPU (serving tests), then C5 over
# HTTP: native front end vs the asyncio server (both with the native batcher)
set -o pipefail
mkdir -p gpurun_out/r5y
timeout -k 10 400 python -u -m pytest tests/test_gpu_native_http.py tests/test_gpu_native_batcher.py tests/test_gpu_server.py tests/test_gpu_c5_serving.py tests/test_gpu_v2.py -v --timeout 150 --timeout-method thread > gpurun_out/r5y/serving_tests.txt 2>&1 || exit 1
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python scripts/bench_serving.py --qps 20000,60000,100000,150000 --duration 5 --warmup 1.5 $BS_ARGS | sed "s/}\$/, \"variant\": \"$label\"}/" >> gpurun_out/r5y/c5.jsonl 2>> gpurun_out/r5y/c5.err
}
for rep in 1 2; do
  BS_ARGS="--workers 1 --io-threads 8" run native_w1_io8 KF_NATIVE_HTTP=1 || exit 2
  BS_ARGS="--workers 2 --io-threads 4" run native_w2_io4 KF_NATIVE_HTTP=1 || exit 3
  BS_ARGS="--workers 8 --io-threads 1" run native_w8_io1 KF_NATIVE_HTTP=1 || exit 4
  BS_ARGS="--workers 8" run asyncio_w8 KF_NATIVE_HTTP=0 || exit 5
done
