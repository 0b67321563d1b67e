# one GPU call of the round: the GPU test suite, the bench, A/B runs, a rocprof summary.
# A failing test does not stop the call; a crash, abort or time limit does.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r4b}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > gpurun_out/${P}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc tests
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.jsonl 2> gpurun_out/${P}_bench.err || exit 2
bash scripts/ab_env.sh TI_COVER_ORDER=0 ${P}_cover c4 c3 c3_maxbin || exit 3
bash scripts/ab_variant.sh t8mask ${P}_mask c3 c3_maxbin || exit 4
bash scripts/ab_variant.sh vbin ${P}_vbin c2 || exit 6
bash scripts/ab_env.sh TI_FIX_PERM=0 ${P}_perm c2 || exit 7
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --configs "" --no-cpu-baseline --latency-qps 0 --host-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/${P}_bench_prof.jsonl 2>&1 || exit 5
