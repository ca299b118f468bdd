#!/bin/bash
# prefill: parity + end-to-end time per (WF_PG_ALG, WF_PF_EPI) pair: CFGS="0:1 0:0 3:1" bash tools/pf_epi_study.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in ${CFGS:-0:0 0:1}; do
  a=${cfg%%:*}; r=${cfg#*:}; e=${r%%:*}; a8=${r#*:}; [ "$a8" = "$r" ] && a8=$a
  echo "== WF_PG_ALG=$a WF_PG_ALG8=$a8 WF_PF_EPI=$e"
  WF_PG_ALG=$a WF_PG_ALG8=$a8 WF_PF_EPI=$e timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "prefill and not study" 2>&1 | tail -1 || exit 1
  WF_PG_ALG=$a WF_PG_ALG8=$a8 WF_PF_EPI=$e timeout -k 10 200 python tools/prefill_bench.py | cut -c1-110 || exit 1
done
