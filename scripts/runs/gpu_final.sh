# round-4 measurement call: TreeSHAP kernels, the bench with every round-4 PMC
# pass in place, and C5 over HTTP with 8 workers
set -o pipefail
P=${1:-r4e}
mkdir -p gpurun_out
timeout -k 10 300 python scripts/shap_bench.py > gpurun_out/${P}_shap.jsonl 2>gpurun_out/${P}_shap.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.jsonl 2> gpurun_out/${P}_bench.err || exit 2
timeout -k 10 300 python scripts/bench_serving.py --workers 8 --qps 20000,40000,60000 --duration 6 > gpurun_out/${P}_c5_w8.jsonl 2> gpurun_out/${P}_c5.err || exit 3
