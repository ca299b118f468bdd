#!/bin/bash
# Same-box A/B of an environment switch on the end-to-end prefill (alternating runs):
# VAR=name VALS="1 0" bash tools/ab_prefill.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in ${VALS:-1 0}; do
    echo -n "$VAR=$v rep $rep: "
    env "$VAR=$v" timeout -k 10 200 python tools/prefill_bench.py --iters 5 | cut -c1-100 || exit 1
  done
done
