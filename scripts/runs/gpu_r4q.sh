# two-stream headline: its GPU test, the default bench line, both rocprof summaries
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_identity.py tests/test_gpu_bench_ranks.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r4q_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4q_bench.jsonl 2> gpurun_out/r4q_bench.err || exit 2
bash scripts/gpu_headline_prof.sh r4q || exit 3
