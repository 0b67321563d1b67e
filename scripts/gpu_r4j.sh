set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bheap.py tests/test_gpu_parity.py -v -rs --timeout 150 --timeout-method thread > gpurun_out/r4j_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/env_sweep.sh r4j_halves c2 "TI_FIX_HALVES=2" || exit 2
bash scripts/env_sweep.sh r4j_halves_hist c2_hist "TI_FIX_HALVES=2" || exit 3
