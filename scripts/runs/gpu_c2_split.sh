# C2 kernel time against the tree count (fixed per-tile cost vs per-tree cost)
set -o pipefail
mkdir -p gpurun_out/r4f
for rep in 1 2; do
  for t in 4 32 125 250 500; do
    timeout -k 10 120 python scripts/kernel_workload.py --workload c2 --trees $t --steps 10 --x-buffers 3 >> gpurun_out/r4f/c2_trees.jsonl || exit 1
  done
done
