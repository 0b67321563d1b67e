# end-of-round validation on one MI355X: the GPU suite, smoke, the bench and a
# kernel-trace summary of the bench command (the driver's own order; the
# profiled run leaves out the HTTP leg, whose server process rocprof would trace too)
set -o pipefail
P=${1:-r4h}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > gpurun_out/${P}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.jsonl 2> gpurun_out/${P}_bench.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${P}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --c5-http-qps "" --c5-http-v2-qps "" > $GRAFT_REPO_ROOT/gpurun_out/${P}_bench_under_rocprof.jsonl 2>&1 || exit 4
