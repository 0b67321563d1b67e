# bench headline (two streams) under engine settings, interleaved, two rounds:
# scripts/streams_env_ab.sh OUT_SUBDIR "A=1" "B=2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for kv in "X=0" "$@"; do
    env $kv timeout -k 10 200 python bench.py --steps 50 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 > $OUT/tmp.json 2>/dev/null || exit 1
    tail -1 $OUT/tmp.json | sed "s/^{/{\"setting\": \"$kv\", /" >> $OUT/ab.jsonl
  done
done
