# C4 hot-prefix cache: parity, then A/B over TI_HX_HOT at 1M rows; PMC passes
# of C3's two bottoms
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_c4_full.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r5j_c4_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for h in 0 16 32 64 80 128; do
    TI_HX_HOT=$h timeout -k 10 120 python scripts/kernel_workload.py --workload c4 --steps 10 | sed "s/}$/, \"variant\": \"TI_HX_HOT=$h\"}/" >> gpurun_out/r5j_c4_hot.jsonl || exit 2
  done
done
TI_TX16=0 bash scripts/kernel_pmc.sh r5i_c3_rec c3 || exit 3
TI_TX16_ILP=8 TI_TX_TOP=8 bash scripts/kernel_pmc.sh r5i_c3_t16 c3 || exit 4
TI_TX16=0 bash scripts/gpu_c3_l2.sh r5i_c3_l2_rec c3 || exit 5
