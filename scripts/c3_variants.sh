#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "TI_FORCE_LAYOUT=explicit" "TI_CPT_FEAT_LDS=1" "TI_CPT_FEAT_LDS=0" "TI_FORCE_LAYOUT=explicit TI_X=1"; do
  out=$(env $v timeout -k 10 300 python scripts/bench_configs.py --configs c3 2>/dev/null | tail -1)
  rc=$?
  echo "$v :: $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3e rows/s kernel %.2f ms layout %d" % (d["rows_per_s"], d["kernel_ms"], d["layout"]))' 2>/dev/null)" | tee -a gpurun_out/c3_variants.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
