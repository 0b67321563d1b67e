#!/bin/bash
# C5 over HTTP as bench.py's c5_http leg runs it (one worker, 16 IO threads,
# 4 load generator threads, 4 s points after 1.5 s of warm-up), two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python scripts/bench_serving.py --qps 20000,100000,200000 --workers 1 \
    --io-threads 16 --loadgen-threads 4 --duration 4 --warmup 1.5 --port $((18100 + rep)) \
    >> gpurun_out/r5ai_c5_http.jsonl 2>> gpurun_out/r5ai_c5_http.err || exit 1
done
