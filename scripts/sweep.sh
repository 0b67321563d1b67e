#!/bin/bash
# Sweep heap-kernel launch knobs on the C2 bench (one process per setting).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rows in ${ROWS_LIST:-256 512}; do
  for kb in ${KB_LIST:-40 53 80}; do
    out=$(TI_HEAP_ROWS=$rows TI_HEAP_LDS_KB=$kb timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)
    rc=$?
    echo "rows=$rows kb=$kb $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3e rows/s  kernel %.3f ms" % (d["value"], d["roofline"]["kernel_ms"]))' 2>/dev/null)" | tee -a gpurun_out/sweep.log
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  done
done
exit 0
