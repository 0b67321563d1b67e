set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bheap.py tests/test_gpu_bench_ranks.py -v -rs --timeout 150 --timeout-method thread > gpurun_out/r4g_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/env_sweep.sh r4g_binq c2 "TI_FIX_BINQ=8" || exit 2
bash scripts/env_sweep.sh r4g_binq_hist c2_hist "TI_FIX_BINQ=8" || exit 3
