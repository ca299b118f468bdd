#!/bin/bash
# prefill GEMM main-loop study: WF_PG_ALG variants (parity of the tiled GEMM and the prefill path,
# standalone GEMM bench, end-to-end prefill)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for a in ${ALGS:-0 1}; do
  echo "== WF_PG_ALG=$a"
  WF_PG_ALG=$a timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "prefill and not study" 2>&1 | tail -2 || exit 1
  WF_PG_ALG=$a timeout -k 10 200 python tools/prefill_gemm_bench.py 2>&1 | grep -v amdgpu.ids | cut -c1-110 || exit 1
  WF_PG_ALG=$a timeout -k 10 200 python tools/prefill_bench.py | cut -c1-110 || exit 1
done
