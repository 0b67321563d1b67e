#!/bin/bash
# GPU suite, bench, C2 PMC passes (incl. HBM counters), FETCH_SIZE calibration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$RUN_TESTS" ] && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1
true
timeout -k 10 300 python3 bench.py > gpurun_out/bench.jsonl 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.jsonl
PMC_HBM=1 scripts/pmc_passes.sh r2_c2 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-qps 0 --nan-variant 0 --configs "" || exit $?
(cd /tmp && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/fetch_calib" -o run --output-format csv -- "$GRAFT_REPO_ROOT/scripts/micro/fetch_calib") > gpurun_out/fetch_calib.log 2>&1
echo "calib rc=$?"
