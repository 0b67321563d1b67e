#!/bin/bash
# Round-2 probe: counter list + rocprofv3 stats/PMC of the C3 explicit kernel (1M rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 120 rocprofv3 -L) > gpurun_out/rocprof_counters.txt 2>&1
echo "counters rc=$?"
timeout -k 10 300 python3 scripts/bench_configs.py --configs c3 --rows3 1000000 --steps 5 > gpurun_out/c3_1m.jsonl 2> gpurun_out/c3_1m.err || exit $?
cat gpurun_out/c3_1m.jsonl
scripts/profile_cmd.sh r2_c3_prof scripts/bench_configs.py --configs c3 --rows3 1000000 --steps 3
