#!/bin/bash
# layouts 6/7 parity subset + explicit sweep (C3, C4); extra args = sweep settings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "every_layout or zero_missing or record_layouts or leafwise" > gpurun_out/lx_tests.log 2>&1
rc=$?; tail -5 gpurun_out/lx_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u scripts/explicit_sweep.py --configs c3 --settings "${1:-rexplicit:16,lexplicit:8,lexplicit:4}" > gpurun_out/lx_sweep.jsonl 2> gpurun_out/lx_sweep.err
rc=$?; cat gpurun_out/lx_sweep.jsonl; tail -3 gpurun_out/lx_sweep.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/explicit_sweep.py --configs c4 --settings "${2:-rexplicit:8,rexplicit:4,rexplicit:16}" >> gpurun_out/lx_sweep.jsonl 2>> gpurun_out/lx_sweep.err
rc=$?; tail -3 gpurun_out/lx_sweep.jsonl; exit $rc
