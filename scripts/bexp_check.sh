#!/bin/bash
# binned-explicit round: gpu tests, then C3/C4 with binned and float explicit kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
step configs_bexp 400 python scripts/bench_configs.py --configs c3,c4
step configs_exp 400 env TI_NO_BEXPLICIT=1 python scripts/bench_configs.py --configs c3
exit 0
