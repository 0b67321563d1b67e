# round 5: C5 over HTTP (8 workers), native batcher against the asyncio
# batcher (KF_NATIVE_BATCHER=0), interleaved, two rounds
set -o pipefail
mkdir -p gpurun_out/r5w
for rep in 1 2; do
  for nb in 1 0; do
    KF_NATIVE_BATCHER=$nb timeout -k 10 200 python scripts/bench_serving.py --workers 8 --qps 20000,40000,60000 --duration 6 | sed "s/}/, \"native_batcher\": $nb}/" >> gpurun_out/r5w/c5_ab.jsonl 2>> gpurun_out/r5w/c5.err || exit 1
  done
done
