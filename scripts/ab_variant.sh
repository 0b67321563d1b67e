cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/kfserving_amd/lib/variants/nt0/libtreeinfer.so
for rep in 1 2; do
for w in c2 c3 c3_maxbin c4; do
  xb=1; [ $w = c2 ] && xb=3
  timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"nt\": 1}/" >> gpurun_out/r3s/ab.jsonl || exit 1
  TREEINFER_LIB=$V timeout -k 10 120 python scripts/kernel_workload.py --workload $w --steps 10 --x-buffers $xb | sed "s/}/, \"nt\": 0}/" >> gpurun_out/r3s/ab.jsonl || exit 1
done; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/r3s/fetch_nt1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/kernel_workload.py --workload c2 --steps 6 --x-buffers 3 > $GRAFT_REPO_ROOT/gpurun_out/r3s/fetch_nt1.log 2>&1
