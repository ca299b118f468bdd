#!/bin/bash
# Same-box prefill A/B: optional parity tests (TESTS) on the product library, then the end-to-end
# prefill bench and the prefill GEMM bench alternated over LIBS (REPS rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abp
mkdir -p "$O"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  eval "timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread -p no:cacheprovider $TESTS" > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
L=$(pwd)/wrinklefree-inference-engine_amd/lib
for rep in $(seq 1 ${REPS:-3}); do
  for lib in ${LIBS:-libwfbitnet.so}; do
    WF_BITNET_LIB=$L/$lib timeout -k 10 300 python tools/prefill_bench.py > "$O/last.log" 2>&1 || { tail -20 "$O/last.log"; exit 1; }
    echo "e2e $lib rep $rep: $(grep workload "$O/last.log" | cut -c1-160)"
    WF_BITNET_LIB=$L/$lib timeout -k 10 300 python tools/prefill_gemm_bench.py > "$O/last.log" 2>&1 || { tail -20 "$O/last.log"; exit 1; }
    echo "gemm $lib rep $rep: $(tail -1 "$O/last.log" | cut -c1-300)"
  done
done
