mkdir -p gpurun_out/r4p
for rep in 1 2; do
  for s in 1 2 3; do
    timeout -k 10 200 python bench.py --steps 50 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 --streams $s > gpurun_out/r4p/s$s.$rep.json 2>gpurun_out/r4p/s$s.$rep.err || exit 1
  done
done
