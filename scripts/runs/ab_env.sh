#!/bin/bash
# A/B of one engine setting read at forest creation (an environment knob such
# as TI_COVER_ORDER=0) against the default, on the kernel workloads of
# scripts/kernel_workload.py, interleaved, two rounds.
# Usage: scripts/ab_env.sh VAR=VALUE OUT_SUBDIR [workloads...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
KV=$1
OUT=gpurun_out/$2
shift 2
mkdir -p "$OUT"
WL=${*:-c2 c3 c3_maxbin c4}
for rep in 1 2; do
  for w in $WL; do
    xb=1; [ "$w" = c2 ] && xb=3
    timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"variant\": 0}/" >> $OUT/ab.jsonl || exit 1
    env "$KV" timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"variant\": \"$KV\"}/" >> $OUT/ab.jsonl || exit 1
  done
done
