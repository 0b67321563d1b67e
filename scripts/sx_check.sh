#!/bin/bash
# Staged binned explicit (layout 5): parity tests on every layout, then C3 with
# layout 5 (default) against layout 4 (TI_NO_SEXPLICIT=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "layout or bexplicit or lgb or sklearn" \
  > gpurun_out/sx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/sx_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "TI_X=0" "TI_NO_SEXPLICIT=1" "TI_SX_ILP=4"; do
  env $v timeout -k 10 300 python scripts/bench_configs.py --configs c3 > gpurun_out/sx_c3_tmp.log 2>&1
  rc=$?
  echo "$v :: $(tail -1 gpurun_out/sx_c3_tmp.log)" | tee -a gpurun_out/sx_c3.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
