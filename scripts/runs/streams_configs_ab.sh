# one stream vs two on the config workloads (scripts/kernel_workload.py), 1M rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for w in ${*:-c2_hist c3 c3_maxbin c4}; do
    for s in 1 2; do
      timeout -k 10 150 python scripts/kernel_workload.py --workload $w --steps 10 --streams $s >> $OUT/ab.jsonl || exit 1
    done
  done
done
