#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench (+ optional rocprof).
# Stops at the first crash-type exit (abort/segfault/timeout); a plain test
# failure (exit 1) still lets the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc $name" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider -rf
step bench 600 python bench.py --steps 20 --warmup 5
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
exit 0
