#!/bin/bash
# Slot-record explicit layouts (5 staged in LDS, 6 global): parity tests on
# every layout, then C3 / C4 against layout 4 (the default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "layout or bexplicit or lgb or sklearn" \
  > gpurun_out/sx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/sx_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "TI_X=0" "TI_FORCE_LAYOUT=gexplicit" "TI_FORCE_LAYOUT=gexplicit TI_SX_ILP=4" "TI_FORCE_LAYOUT=gexplicit TI_SX_ILP=8"; do
  env $v timeout -k 10 300 python scripts/bench_configs.py --configs ${CFGS:-c3,c4} > gpurun_out/sx_tmp.log 2>&1
  rc=$?
  echo "$v :: $(grep rows_per_s gpurun_out/sx_tmp.log | python -c 'import sys,json; [print("%s %.3e rows/s kernel %.2f ms layout %d" % (d["config"][:3], d["rows_per_s"], d["kernel_ms"], d["layout"])) for d in map(json.loads, sys.stdin)]')" | tee -a gpurun_out/sx_cfg.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
