#!/bin/bash
# C3 (and optionally C4) across variant libraries: scripts/sweep_configs.sh "c3" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cfg=$1; shift
for n in "$@"; do
  if [ "$n" = default ]; then lib=kfserving_amd/lib/libtreeinfer.so; else lib=kfserving_amd/lib/variants/libtreeinfer_$n.so; fi
  r=$(timeout -k 10 300 env TREEINFER_LIB=$lib ${SWEEP_ENV} python scripts/bench_configs.py --configs $cfg 2>/dev/null | python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{"):
        d=json.loads(l); print("%s %.4e rows/s kernel %.3f ms layout %s;" % (d["config"][:2], d["rows_per_s"], d["kernel_ms"], d["layout"]), end=" ")')
  echo "$n ${SWEEP_ENV} :: $r" | tee -a gpurun_out/sweep.log
done
