cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_lat.log 2>&1 || exit $?
for v in "TI_FORCE_LAYOUT=explicit" "TI_FORCE_LAYOUT=compact"; do
  env $v timeout -k 10 300 python scripts/bench_configs.py --configs c3 --f3 28 2>/dev/null | tail -1 | sed "s/^/$v /" >> gpurun_out/c3_f28.log || exit $?
done
exit 0
