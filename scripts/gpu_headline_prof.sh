# rocprofv3 kernel-trace summary of the headline alone (warm-up + timed steps
# of the C2 kernel, no other legs), whose average must agree with the bench
# line's event-timed kernel_ms
set -o pipefail
P=${1:-r4i}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 > $GRAFT_REPO_ROOT/gpurun_out/${P}_headline_under_rocprof.jsonl 2>&1 || exit 1
