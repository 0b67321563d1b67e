set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rs --timeout 200 --timeout-method thread > gpurun_out/r4a_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench.jsonl 2> gpurun_out/r4a_bench.err || exit 2
bash scripts/ab_variant.sh t8mask r4a_ab c3 c3_maxbin c3_f64 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/r4a_bench_prof.jsonl 2>&1 || exit 4
