#!/bin/bash
# Build the working tree's library with extra study defines for same-box A/B runs:
#   bash tools/build_var.sh NAME "-DWF_X -DWF_Y"  ->  wrinklefree-inference-engine_amd/lib/libwfbitnet_NAME.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; DEFS=${2:-}
T=$(mktemp -d)
C=wrinklefree-inference-engine_amd/csrc
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-result -Iinclude -I$C $DEFS"
pids=()
for f in wf_gemv wf_attn wf_decode wf_mfma wf_msb; do
  /opt/rocm/bin/hipcc $FL -c "$C/$f.hip" -o "$T/$f.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "wrinklefree-inference-engine_amd/lib/libwfbitnet_$NAME.so" "$T"/*.o
rm -rf "$T"
echo "built lib/libwfbitnet_$NAME.so with '$DEFS'"
