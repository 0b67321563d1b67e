# round 5: c3_maxbin's compact u8 bottom at 2 / 3 / 4 trees a lane (bit-exact
# tests at 2 and 3, then an interleaved A/B at 1M rows), and C5 over HTTP with
# the native batcher (8 workers)
set -o pipefail
mkdir -p gpurun_out/r5v
for ilp in 2 3; do
  TI_LX_ILP=$ilp timeout -k 10 300 python -u -m pytest tests/test_gpu_u8_bins.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5v/u8_tests_ilp$ilp.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for ilp in 4 2 3; do
    TI_LX_ILP=$ilp timeout -k 10 120 python scripts/kernel_workload.py --workload c3_maxbin --steps 10 | sed "s/}/, \"ilp\": $ilp}/" >> gpurun_out/r5v/c3_maxbin_ilp.jsonl || exit 2
  done
done
timeout -k 10 300 python scripts/bench_serving.py --workers 8 --qps 20000,40000,60000 --duration 6 > gpurun_out/r5v/c5_w8.jsonl 2> gpurun_out/r5v/c5.err || exit 3
