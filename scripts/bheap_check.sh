#!/bin/bash
# binned-heap round: gpu tests, then bench with the binned (default) and the
# float-compare heap kernels side by side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a gpurun_out/steps.log
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step bheap_tests 300 python -u -m pytest tests/test_gpu_bheap.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
step bench_bheap 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-qps 0
step bench_heap 300 env TI_NO_BHEAP=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-qps 0
exit 0
