#!/bin/bash
# Round-2 re-profile after the fused-leaf C2 step and layouts 8 / 9: C2 PMC
# passes over bench.py (HBM counters included), then the C3 (layout 9) and C4
# (layout 8) passes of scripts/r2_cfgprof.sh, and rocprofv3 --stats of the
# default bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC_HBM=1 scripts/pmc_passes.sh r2b_c2 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-qps 0 --nan-variant 0 --configs "" --host-rows 0 || exit $?
bash scripts/r2_cfgprof.sh r2b_c3_l9 c3 texplicit:7 r2b_c4_l8 c4 hexplicit:8 || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2b_bench_stats" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline) > gpurun_out/r2b_bench_stats.log 2>&1
echo "bench stats rc=$?"
