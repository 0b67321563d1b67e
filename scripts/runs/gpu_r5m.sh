# (1) C4 hot-prefix cache with the select deferred (variant hot3): parity, A/B
# (2) t16 per-tree skip (in-tree lib) against no skip (variant hot2): parity, sweep
set -o pipefail
V3=$(pwd)/kfserving_amd/lib/variants/hot3/libtreeinfer.so
V2=$(pwd)/kfserving_amd/lib/variants/hot2/libtreeinfer.so
TREEINFER_LIB=$V3 timeout -k 10 300 python -u -m pytest tests/test_gpu_c4_full.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r5m_c4_tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_u8_bins.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r5m_parity_tests.txt 2>&1 || exit 2
for i in 1 2; do
  for h in 0 16 32 64; do
    TREEINFER_LIB=$V3 TI_HX_HOT=$h timeout -k 10 120 python scripts/kernel_workload.py --workload c4 --steps 10 | sed "s/}$/, \"variant\": \"hot3 TI_HX_HOT=$h\"}/" >> gpurun_out/r5m_c4_hot.jsonl || exit 3
  done
  for v in skip noskip; do
    L=$(pwd)/kfserving_amd/lib/libtreeinfer.so; [ $v = noskip ] && L=$V2
    for cfg in "8 8" "8 6" "4 6" "12 6" "8 7"; do
      set -- $cfg
      TREEINFER_LIB=$L TI_TX16_ILP=$1 TI_TX_TOP=$2 timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --steps 5 | sed "s/}$/, \"variant\": \"$v ilp$1 top$2\"}/" >> gpurun_out/r5m_c3_skip.jsonl || exit 4
    done
  done
  TI_TX16=0 timeout -k 10 120 python scripts/kernel_workload.py --workload c3 --steps 5 | sed "s/}$/, \"variant\": \"records\"}/" >> gpurun_out/r5m_c3_skip.jsonl || exit 5
done
