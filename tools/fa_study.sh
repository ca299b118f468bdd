for v in ${VARS:-0 11 12}; do echo "== $v"; WF_PF_ATTN=$v timeout -k 10 120 python tools/prefill_bench.py | cut -c1-120 || exit 1; done
