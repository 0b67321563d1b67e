# one stream vs two at large batches (20M rows; C4 10M), interleaved, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
for rep in 1 2; do
  for w in c3 c3_maxbin c4; do
    r=20000000; [ $w = c4 ] && r=10000000
    for s in 1 2; do
      timeout -k 10 200 python scripts/kernel_workload.py --workload $w --rows $r --steps 6 --streams $s >> $OUT/ab.jsonl || exit 1
    done
  done
done
