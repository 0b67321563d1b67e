#!/bin/bash
# Build a variant of libtreeinfer.so with extra compile-time knobs, for A/B
# runs through TREEINFER_LIB.  Usage: scripts/build_variant.sh NAME "-DTI_TILP=16 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
FLAGS="$*"
OUT=kfserving_amd/lib/variants/$NAME
mkdir -p "$OUT"
CF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -fno-gpu-flush-denormals-to-zero -Iinclude -Ikfserving_amd/csrc $FLAGS"
pids=()
for u in treeinfer treeinfer_k_ff treeinfer_k_fd treeinfer_k_dd treeinfer_k_df; do
  /opt/rocm/bin/hipcc $CF -c kfserving_amd/csrc/$u.hip -o "$OUT/$u.o" 2> "$OUT/$u.err" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fno-gpu-rdc "$OUT"/*.o -o "kfserving_amd/lib/variants/libtreeinfer_$NAME.so"
rm -f "$OUT"/*.o
echo "built kfserving_amd/lib/variants/libtreeinfer_$NAME.so"
