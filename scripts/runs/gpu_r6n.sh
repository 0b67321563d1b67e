#!/bin/bash
# C2 fixed walk, 8 trees a lane (TI_BHEAP_NG=3: 8-tree stages walked as one
# group, 3 workgroups a CU) against 4 (NG=1, the default; NG=2: 8-tree stages
# as two groups): interleaved in one process, then the fixed-walk tests with NG=3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TI_DEV_KNOBS=1 TI_OCC=1
timeout -k 10 200 python scripts/runs/c2_ab.py --settings "NG=1;NG=3;NG=2" --rounds 7 > gpurun_out/r6n_c2_gw8_ab.jsonl 2> gpurun_out/r6n_c2_gw8_ab.err || exit 1
timeout -k 10 200 python scripts/runs/c2_ab.py --settings "NG=1;NG=3" --rounds 5 --nan 0.01 >> gpurun_out/r6n_c2_gw8_ab.jsonl 2>> gpurun_out/r6n_c2_gw8_ab.err || exit 1
TI_BHEAP_NG=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_bheap.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n_gw8_tests.txt 2>&1 || exit 2
