#!/bin/bash
# layout-6 parity subset + explicit sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "rexplicit or depth16 or every_layout" > gpurun_out/rx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rx_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/explicit_sweep.py > gpurun_out/rx_sweep.jsonl 2> gpurun_out/rx_sweep.err
rc=$?; cat gpurun_out/rx_sweep.jsonl; tail -3 gpurun_out/rx_sweep.err; exit $rc
