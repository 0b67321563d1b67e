#!/bin/bash
# C5 over HTTP on one GPU: does the p99 tail at a fixed offered rate depend on
# the measuring window (4 s, the bench's, vs 10 s) and on being the first
# point after the server starts?  20k / 100k / 200k / 20k req/s, one worker,
# 16 IO threads, 4,096 connections, 4 load-generator threads; two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for dur in 4 10; do
    timeout -k 10 200 python scripts/bench_serving.py --qps 20000,100000,200000,20000 --workers 1 \
      --io-threads 16 --loadgen-threads 4 --duration $dur --warmup 1.5 --port $((18200 + rep * 10 + dur)) \
      | sed "s/}$/, \"window_s\": $dur, \"rep\": $rep}/" >> gpurun_out/r6r_c5_window.jsonl || exit 1
  done
done
