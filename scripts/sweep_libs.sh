#!/bin/bash
# A/B the C2 bench across variant libraries (scripts/build_variant.sh).
# Usage: scripts/sweep_libs.sh name1 name2 ...   ("default" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "$@"; do
  if [ "$n" = default ]; then lib=kfserving_amd/lib/libtreeinfer.so; else lib=kfserving_amd/lib/variants/libtreeinfer_$n.so; fi
  r=$(timeout -k 10 120 env TREEINFER_LIB=$lib ${SWEEP_ENV} python bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-qps 0 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e rows/s kernel %.4f ms layout %s" % (d["value"], d["roofline"]["kernel_ms"], d["config"]["layout"]))')
  echo "$n ${SWEEP_ENV} :: $r" | tee -a gpurun_out/sweep.log
done
