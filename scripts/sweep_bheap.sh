#!/bin/bash
# stage-size sweep of the binned heap kernel on the C2 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in 8 16 24 32; do
  echo "TI_BHEAP_STAGE=$s :: $(timeout -k 10 120 env TI_BHEAP_STAGE=$s python bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-qps 0 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3e rows/s kernel %.3f ms" % (d["value"], d["roofline"]["kernel_ms"]))')" | tee -a gpurun_out/sweep.log
done
