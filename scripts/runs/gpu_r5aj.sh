#!/bin/bash
# C3 at 320-row tiles (2.5 waves per SIMD): the NP2 parity test, then an
# interleaved sweep against the default 256-row tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "np2 or leafwise or heap_top" > gpurun_out/r5aj_tests.txt 2>&1 || exit 1
TI_OCC=1 timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --steps 3 > gpurun_out/r5aj_occ.txt 2>&1
TI_OCC=1 TI_RX_ROWS=320 TI_TX16_ILP=4 timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --steps 3 >> gpurun_out/r5aj_occ.txt 2>&1 || exit 2
bash scripts/env_sweep.sh r5aj c3 "TI_RX_ROWS=320 TI_TX16_ILP=4" "TI_RX_ROWS=320 TI_TX16_ILP=4 TI_TX_TOP=6" "TI_RX_ROWS=320 TI_TX16_ILP=8 TI_TX_TOP=5" "TI_RX_ROWS=320 TI_TX16_ILP=8 TI_TX_TOP=4" "TI_RX_ROWS=320 TI_TX16_ILP=8"
