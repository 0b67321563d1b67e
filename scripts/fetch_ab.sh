#!/bin/bash
# FETCH_SIZE (one --pmc pass, kernel-trace only) + timing of the C2 bench per
# variant library.  Usage: scripts/fetch_ab.sh name1 name2 ... ("default" = in-tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/fetch_ab
for n in "$@"; do
  if [ "$n" = default ]; then lib=$ROOT/kfserving_amd/lib/libtreeinfer.so; else lib=$ROOT/kfserving_amd/lib/variants/libtreeinfer_$n.so; fi
  export TREEINFER_LIB=$lib
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/gpurun_out/fetch_ab/$n" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --latency-qps 0 --nan-variant 0) > "$ROOT/gpurun_out/fetch_ab/$n.log" 2>&1 || { echo "$n failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/fetch_ab/$n" "$n" <<'PY'
import csv, glob, sys, json
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/*counter_collection.csv")
     for r in csv.DictReader(open(f)) if "predict_kernel" in r["Kernel_Name"]]
print(sys.argv[2], "FETCH_SIZE x2 MB per dispatch: %.1f (n=%d)" % (2 * 1024 * sum(v) / len(v) / 1e6, len(v)))
PY
  tail -1 "$ROOT/gpurun_out/fetch_ab/$n.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("  %.4e rows/s kernel %.4f ms" % (d["value"], d["roofline"]["kernel_ms"]))'
done
