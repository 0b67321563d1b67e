#!/bin/bash
# A/B library builds (TREEINFER_LIB) on the C2 bench; interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for lib in ${LIBS:-libtreeinfer.so}; do
    out=$(TREEINFER_LIB=$PWD/kfserving_amd/lib/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)
    rc=$?
    echo "round=$round lib=$lib $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3e rows/s  kernel %.3f ms" % (d["value"], d["roofline"]["kernel_ms"]))' 2>/dev/null)" | tee -a gpurun_out/sweep_libs.log
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  done
done
exit 0
