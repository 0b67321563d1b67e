# rocprofv3 kernel-trace summaries of the headline alone (no other legs).
# 1) --streams 1: every launch alone on the chip; the C2 kernel's average
#    duration must agree with the bench line's event-timed kernel_ms.
# 2) --streams 2 (the default headline): the kernel trace of two batches in
#    flight, to show where consecutive launches overlap.
set -o pipefail
P=${1:-r4i}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 --streams 1 > $GRAFT_REPO_ROOT/gpurun_out/${P}_headline_under_rocprof.jsonl 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --nan-variant 0 --streams 2 > $GRAFT_REPO_ROOT/gpurun_out/${P}_headline2_under_rocprof.jsonl 2>&1 || exit 2
