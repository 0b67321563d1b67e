#!/bin/bash
# native V2 tensor route: GPU tests, then C5 over HTTP with V2 FP32 JSON
# tensor bodies through the native front end (one worker, 16 IO threads, 4
# load generator threads) and through the asyncio server
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_http.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r5as_tests.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_serving.py --protocol v2 --qps 20000,100000,200000 --workers 1 \
  --io-threads 16 --loadgen-threads 4 --duration 4 --warmup 1.5 --port 18120 > gpurun_out/r5as_v2_native.jsonl 2> gpurun_out/r5as_v2_native.err || exit 2
KF_NATIVE_HTTP=0 timeout -k 10 200 python scripts/bench_serving.py --protocol v2 --qps 20000,60000 --workers 8 \
  --loadgen-threads 4 --duration 4 --warmup 1.5 --port 18130 > gpurun_out/r5as_v2_asyncio.jsonl 2> gpurun_out/r5as_v2_asyncio.err || exit 3
