# round 5: serving GPU tests, then the native front end's capacity with a
# 4-thread load generator (the one-thread one stopped near 140k req/s)
set -o pipefail
mkdir -p gpurun_out/r5ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_native_http.py tests/test_gpu_native_batcher.py tests/test_gpu_server.py tests/test_gpu_c5_serving.py -v --timeout 150 --timeout-method thread > gpurun_out/r5ab/serving_tests.txt 2>&1 || exit 1
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 240 python scripts/bench_serving.py --duration 4 --warmup 1.5 --loadgen-threads 4 $BS_ARGS | sed "s/}\$/, \"variant\": \"$label\"}/" >> gpurun_out/r5ab/c5.jsonl 2>> gpurun_out/r5ab/c5.err
}
for rep in 1 2; do
  BS_ARGS="--workers 1 --io-threads 8 --qps 100000,150000,200000,250000,300000" run native_w1_io8 KF_NATIVE_HTTP=1 || exit 2
  BS_ARGS="--workers 1 --io-threads 16 --qps 150000,200000,250000,300000" run native_w1_io16 KF_NATIVE_HTTP=1 || exit 3
  BS_ARGS="--workers 8 --qps 60000,100000,150000" run asyncio_w8 KF_NATIVE_HTTP=0 || exit 4
done
