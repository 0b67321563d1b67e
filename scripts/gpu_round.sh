# one GPU call of the round: the GPU test suite, the bench, then PMC passes of
# the named workloads, then the headline alone (one stream, no other legs)
# under rocprofv3 --kernel-trace --stats, whose average the line's kernel_ms
# must match.  A failing test does not stop the call; a crash, abort
# or time limit does.  Usage: bash scripts/gpu_round.sh PREFIX [pmc workloads...]
set -o pipefail
mkdir -p gpurun_out
P=${1:-r4c}; shift
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > gpurun_out/${P}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc tests
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.jsonl 2> gpurun_out/${P}_bench.err || exit 2
[ $# -gt 0 ] && { bash scripts/gpu_pmc.sh $P "$@" || exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 --host-rows-configs 0 --nan-variant 0 --no-tree-shard --streams 1 --c5-http-qps "" --c5-http-v2-qps "" > $GRAFT_REPO_ROOT/gpurun_out/${P}_bench_prof.jsonl 2>&1 || exit 5
