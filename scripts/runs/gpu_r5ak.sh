#!/bin/bash
# after the 320-row experiment's removal: C3's kernel time on the rebuilt
# library, then the C5-over-HTTP points twice (scripts/gpu_r5ai.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --steps 10 >> gpurun_out/r5ak_c3.jsonl 2>> gpurun_out/r5ak_c3.err || exit 1
done
bash scripts/gpu_r5ai.sh
