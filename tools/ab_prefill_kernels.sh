#!/bin/bash
# Same-box per-kernel prefill A/B: rocprofv3 kernel stats of tools/prefill_bench.py for each library
# in LIBS (kernel tables under gpurun_out/abk/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); O=$R/gpurun_out/abk
mkdir -p "$O"
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-1}); do
  for lib in ${LIBS:-libwfbitnet.so}; do
    cd /tmp && WF_BITNET_LIB=$R/wrinklefree-inference-engine_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/p" -o run -- \
        python3 "$R/tools/prefill_bench.py" --iters 2 > "$O/p.log" 2>&1 || { tail -20 "$O/p.log"; exit 1; }
    cd "$R" && python3 tools/prof_summary.py "$O/p" > "$O/k_${lib%.so}_$rep.txt" 2>&1 || exit 1
    rm -rf "$O/p"
    echo "== $lib rep $rep"; head -9 "$O/k_${lib%.so}_$rep.txt" | cut -c1-120
  done
done
