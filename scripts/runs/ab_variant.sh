#!/bin/bash
# A/B of the in-tree library against a variant build (TREEINFER_LIB) on the
# kernel workloads of scripts/kernel_workload.py, interleaved, two rounds.
# Build the variant with extra -D flags into kfserving_amd/lib/variants/NAME/
# (python scripts/build_variant.py NAME -DFLAG=V ...)
# (git-ignored), then: scripts/ab_variant.sh NAME OUT_SUBDIR [workloads...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$(pwd)/kfserving_amd/lib/variants/$1/libtreeinfer.so
OUT=gpurun_out/$2
shift 2
mkdir -p "$OUT"
WL=${*:-c2 c3 c3_maxbin c4}
for rep in 1 2; do
  for w in $WL; do
    xb=1; [ "$w" = c2 ] && xb=3
    timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"variant\": 0}/" >> $OUT/ab.jsonl || exit 1
    TREEINFER_LIB=$V timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"variant\": 1}/" >> $OUT/ab.jsonl || exit 1
  done
done
