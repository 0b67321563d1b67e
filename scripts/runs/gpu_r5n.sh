# t16 defaults (8 a lane, top 8) and the per-lane-progress walk: parity, then
# an interleaved A/B on C3 / C3-f64 at 1M rows against the record bottom
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_t16.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5n_t16_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for wl in c3 c3_f64; do
    for v in "records TI_TX16=0" "t16 TI_TX16=1" "perlane TI_TX16_PERLANE=1"; do
      set -- $v
      env $2 timeout -k 10 120 python scripts/kernel_workload.py --workload $wl --steps 5 | sed "s/}$/, \"variant\": \"$1\"}/" >> gpurun_out/r5n_ab.jsonl || exit 2
    done
  done
done
