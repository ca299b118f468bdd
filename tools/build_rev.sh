#!/bin/bash
# Build the library of a git revision as a study variant for same-box A/B runs:
#   bash tools/build_rev.sh REV NAME  ->  wrinklefree-inference-engine_amd/lib/libwfbitnet_NAME.so
set -eu
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
T=$(mktemp -d)
git archive "$REV" wrinklefree-inference-engine_amd/csrc include | tar -x -C "$T"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-result -I$T/include -I$T/wrinklefree-inference-engine_amd/csrc"
pids=()
for f in wf_gemv wf_attn wf_decode wf_mfma wf_msb; do
  /opt/rocm/bin/hipcc $FL -c "$T/wrinklefree-inference-engine_amd/csrc/$f.hip" -o "$T/$f.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
mkdir -p wrinklefree-inference-engine_amd/lib
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "wrinklefree-inference-engine_amd/lib/libwfbitnet_$NAME.so" "$T"/*.o
rm -rf "$T"
echo "built lib/libwfbitnet_$NAME.so from $REV"
