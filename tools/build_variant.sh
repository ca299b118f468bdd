#!/bin/bash
# Study build of the library with extra compile flags, for same-box A/B runs (WF_BITNET_LIB=...):
#   bash tools/build_variant.sh NAME -DFLAG=VALUE ...  ->  wrinklefree-inference-engine_amd/lib/libwfbitnet_NAME.so
# Never the product library (lib/libwfbitnet.so is built by the Makefile / __graft_entry__.build()).
set -eu
cd "$(dirname "$0")/../wrinklefree-inference-engine_amd"
NAME=$1; shift
B=build/var_$NAME
mkdir -p "$B" lib
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-result -I../include -Icsrc $*"
pids=()
for f in csrc/wf_gemv.hip csrc/wf_attn.hip csrc/wf_decode.hip csrc/wf_mfma.hip csrc/wf_msb.hip; do
  /opt/rocm/bin/hipcc $FL -c "$f" -o "$B/$(basename "${f%.hip}").o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "lib/libwfbitnet_$NAME.so" "$B"/*.o
echo "built lib/libwfbitnet_$NAME.so"
