set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5f_pipeline_tests.txt 2>&1 || exit 1
bash scripts/gpu_t16_sweep.sh r5f c3 || exit 2
bash scripts/ab_variant.sh bcast r5g_bcast c3_maxbin c3 || exit 3
bash scripts/gpu_c3_l2.sh r5h_c3_l2 c3 || exit 4
