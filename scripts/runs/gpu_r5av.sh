#!/bin/bash
# C5 over HTTP A/B on one box: the current serving build against the r5ar one
# (worktree ab_old/, same kernels), interleaved, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
for rep in 1 2; do
  for tree in new old; do
    d=$ROOT; [ $tree = old ] && d=$ROOT/ab_old
    (cd $d && timeout -k 10 200 python scripts/bench_serving.py --qps 20000,100000,200000 --workers 1 \
      --io-threads 16 --loadgen-threads 4 --duration 4 --warmup 1.5 --port $((18200 + rep * 10)) ) \
      | sed "s/}$/, \"tree\": \"$tree\"}/" >> gpurun_out/r5av_ab.jsonl || exit 1
  done
done
