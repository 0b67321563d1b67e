#!/bin/bash
# C2 kernel only (no CPU baseline, latency leg, C3/C4 or host pipeline), N runs:
# scripts/c2_quick.sh [N] [extra bench.py args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=${1:-2}; shift
for i in $(seq "$n"); do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-qps 0 \
    --configs "" --host-rows 0 "$@" 2> gpurun_out/c2_quick.err > gpurun_out/c2_quick.json || { tail -5 gpurun_out/c2_quick.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c2_quick.json')); print(json.dumps({'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'nan_rows_per_s': d.get('nan_variant', {}).get('rows_per_s')}))"
done
