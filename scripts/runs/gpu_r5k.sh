# C4 hot-prefix cache, branch-free step (variant hot2): parity, then A/B over TI_HX_HOT
set -o pipefail
V=$(pwd)/kfserving_amd/lib/variants/hot2/libtreeinfer.so
TREEINFER_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_c4_full.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r5k_c4_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for h in 0 16 32 64; do
    TREEINFER_LIB=$V TI_HX_HOT=$h timeout -k 10 120 python scripts/kernel_workload.py --workload c4 --steps 10 | sed "s/}$/, \"variant\": \"hot2 TI_HX_HOT=$h\"}/" >> gpurun_out/r5k_c4_hot.jsonl || exit 2
  done
done
