# round 5: the serving GPU tests through the native batcher's converting
# submit, then C5 over HTTP (8 workers) native vs asyncio batcher, interleaved
set -o pipefail
mkdir -p gpurun_out/r5x
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_batcher.py tests/test_gpu_server.py tests/test_gpu_c5_serving.py tests/test_gpu_v2.py -v --timeout 150 --timeout-method thread > gpurun_out/r5x/serving_tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for nb in 1 0; do
    KF_NATIVE_BATCHER=$nb timeout -k 10 200 python scripts/bench_serving.py --workers 8 --qps 20000,40000,60000,80000 --duration 6 | sed "s/\}\$/, \"native_batcher\": $nb}/" >> gpurun_out/r5x/c5_ab.jsonl 2>> gpurun_out/r5x/c5.err || exit 2
  done
done
