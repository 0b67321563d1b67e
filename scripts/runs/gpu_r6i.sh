# round 6: layout 9's u8 bottom walked two lanes a row -- its tests, then an
# interleaved A/B against the one-lane walk (c3_maxbin at 1M rows; the split
# walk with stages sized for 2 and 3 workgroups a CU)
set -o pipefail
mkdir -p gpurun_out
export TI_DEV_KNOBS=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_u8_bins.py -v --timeout 150 --timeout-method thread > gpurun_out/r6i_u8_tests.txt 2>&1
rc=$?; echo "u8 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
for r in 1 2; do
  for v in "TI_TX8_SPLIT=1" "TI_TX8_SPLIT=1 TI_LX_WGS=3" "TI_TX8_SPLIT=0"; do
    env $v timeout -k 10 180 python scripts/kernel_workload.py --workload c3_maxbin --steps 5 | sed "s/^{/{\"env\": \"$v\", /" >> gpurun_out/r6i_u8_split_ab.jsonl || exit 3
  done
done
