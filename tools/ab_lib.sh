#!/bin/bash
# Same-box A/B of two builds of the library on the end-to-end prefill (alternating runs):
# LIBS="libwfbitnet.so libwfbitnet_prev.so" bash tools/ab_lib.sh [prefill_bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$(pwd)/wrinklefree-inference-engine_amd/lib
for rep in 1 2; do
  for lib in ${LIBS:-libwfbitnet.so libwfbitnet_prev.so}; do
    echo -n "$lib rep $rep: "
    WF_BITNET_LIB=$L/$lib timeout -k 10 200 python tools/prefill_bench.py --iters 5 "$@" | cut -c1-100 || exit 1
  done
done
