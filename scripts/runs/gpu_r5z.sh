# round 5: C5 over HTTP after the native front end's connection balancing:
# native front end (workers x IO threads) against the asyncio server
set -o pipefail
mkdir -p gpurun_out/r5z
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 240 python scripts/bench_serving.py --qps 20000,60000,100000,150000,200000 --duration 4 --warmup 1.5 $BS_ARGS | sed "s/}\$/, \"variant\": \"$label\"}/" >> gpurun_out/r5z/c5.jsonl 2>> gpurun_out/r5z/c5.err
}
for rep in 1 2; do
  BS_ARGS="--workers 1 --io-threads 8" run native_w1_io8 KF_NATIVE_HTTP=1 || exit 2
  BS_ARGS="--workers 2 --io-threads 4" run native_w2_io4 KF_NATIVE_HTTP=1 || exit 3
  BS_ARGS="--workers 4 --io-threads 4" run native_w4_io4 KF_NATIVE_HTTP=1 || exit 4
  BS_ARGS="--workers 8" run asyncio_w8 KF_NATIVE_HTTP=0 || exit 5
done
