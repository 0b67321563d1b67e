# the tree-sharded bench leg: GPU rank tests, then the bench's line at N = 1
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_tree_shard.py tests/test_gpu_bench_identity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5s_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 > gpurun_out/r5s_bench.jsonl 2> gpurun_out/r5s_bench.err || exit 2
