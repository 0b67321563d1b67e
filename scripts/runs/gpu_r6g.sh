# round 6: the two-lanes-a-row C3 walk after the scalar position-table fix --
# its tests, an interleaved A/B against the one-lane walk, then PMC passes
set -o pipefail
mkdir -p gpurun_out
export TI_DEV_KNOBS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_t16.py -v --timeout 150 --timeout-method thread > gpurun_out/r6g_t16_tests.txt 2>&1
rc=$?; echo "t16 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
for r in 1 2; do for v in 1 0; do for w in c3 c3_f64; do
  TI_TX16_SPLIT=$v timeout -k 10 180 python scripts/kernel_workload.py --workload $w --steps 5 >> gpurun_out/r6g_split_ab.jsonl || exit 3
done; done; done
bash scripts/gpu_pmc.sh r6g c3 c3_f64 || exit 4
