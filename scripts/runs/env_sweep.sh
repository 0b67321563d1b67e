#!/bin/bash
# Interleaved sweep of engine settings read at forest creation, on one kernel
# workload of scripts/kernel_workload.py: the default and every setting, two
# rounds.  Usage: scripts/env_sweep.sh OUT_SUBDIR WORKLOAD "A=1 B=2" "A=3" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; W=$2; shift 2
mkdir -p "$OUT"
xb=1; [ "$W" = c2 ] && xb=3
for rep in 1 2; do
  timeout -k 10 120 python scripts/kernel_workload.py --workload $W --steps 10 --x-buffers $xb | sed "s/}/, \"setting\": \"default\"}/" >> $OUT/sweep.jsonl || exit 1
  for kv in "$@"; do
    env $kv timeout -k 10 120 python scripts/kernel_workload.py --workload $W --steps 10 --x-buffers $xb | sed "s/}/, \"setting\": \"$kv\"}/" >> $OUT/sweep.jsonl || exit 1
  done
done
