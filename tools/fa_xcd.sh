#!/bin/bash
# prefill attention XCD-chunked order A/B (parity + end to end): bash tools/fa_xcd.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for x in ${XS:-1 0}; do
  echo "== WF_PF_XCD=$x"
  WF_PF_XCD=$x timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "prefill" 2>&1 | tail -1 || exit 1
  WF_PF_XCD=$x timeout -k 10 200 python tools/prefill_bench.py | cut -c1-110 || exit 1
  WF_PF_XCD=$x timeout -k 10 200 python tools/prefill_bench.py --paged | cut -c1-110 || exit 1
done
