#!/bin/bash
# Round 5: the compact u16 bottom (t16explicit) -- parity of the explicit
# layouts first, then an interleaved A/B against the record bottom on C3 /
# C3-f64 at 1M rows.  Usage: bash scripts/gpu_t16.sh PREFIX
set -o pipefail
P=${1:-r5b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_u8_bins.py tests/test_gpu_many_groups.py -x -v -rs --timeout 150 --timeout-method thread > gpurun_out/${P}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    for wl in c3 c3_f64; do
      TI_TX16=$v timeout -k 10 120 python scripts/kernel_workload.py --workload $wl --steps 5 | sed "s/}$/, \"variant\": \"TI_TX16=$v\"}/" >> gpurun_out/${P}_t16_ab.jsonl || exit 2
    done
  done
done
