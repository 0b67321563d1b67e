#!/bin/bash
# C3 float32's host path runs 64 MB chunks (167,424 rows): the kernel's time
# at that batch size, one stream and two (the pipeline's two lanes), against
# 1M rows; and the host leg at 64 / 256 MB chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/r6s_c3_chunk.jsonl
for rows in 167424 334848 669696 1000000; do
  for s in 1 2; do
    timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --rows $rows --streams $s --steps 10 >> $O || exit 1
  done
done
for mb in 64 256; do
  TI_CHUNK_MB=$mb timeout -k 10 200 python bench.py --steps 2 --warmup 1 --configs c3 --rows3 8000000 --config-steps 1 \
    --no-cpu-baseline --latency-qps 0 --host-rows 0 --host-rows-configs 8000000 --nan-variant 0 --no-tree-shard \
    --streams 1 --c5-http-qps "" --c5-http-v2-qps "" | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print(json.dumps({'chunk_mb': $mb, **d['host_pipeline_c3']}))" >> $O || exit 2
done
