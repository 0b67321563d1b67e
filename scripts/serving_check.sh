#!/bin/bash
# C5 serving runs on one GPU: 4096 connections, open-loop QPS sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ulimit -n "$(ulimit -Hn)" 2>/dev/null
echo "nofile $(ulimit -n)" > gpurun_out/serving.log
timeout -k 10 400 python scripts/bench_serving.py --model c2 --workers "${WORKERS:-4}" --conns 4096 \
  --qps "${QPS:-5000,10000,20000,40000}" --duration 8 --warmup 2 >> gpurun_out/serving.log 2>&1
rc=$?
tail -6 gpurun_out/serving.log
exit $rc
