# bench.py's host_pipeline leg (pageable numpy -> numpy, C2) under engine
# settings, interleaved, two rounds: scripts/host_pipeline_ab.sh OUT "A=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for kv in "X=0" "$@"; do
    env $kv timeout -k 10 200 python bench.py --steps 5 --warmup 2 --configs "" --no-cpu-baseline --latency-qps 0 --nan-variant 0 > $OUT/tmp.json 2>/dev/null || exit 1
    tail -1 $OUT/tmp.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['host_pipeline']; h['setting']='$kv'; print(json.dumps(h))" >> $OUT/ab.jsonl || exit 1
  done
done
