#!/bin/bash
# Same-box A/B of prefill attention variants: parity prints (8 x 2048 full width, kernel vs oracle) and
# the prefill kernel stats per library.
#   VAR="name [name2 ...]" [NOTEST=1] bash tools/ab_prefill.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for L in product $VAR; do
  if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
  if [ -z "${NOTEST:-}" ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -s --timeout 500 --timeout-method thread -p no:cacheprovider \
      -k "prefill_8x2048 or prefill_attention_vs_oracle" > $O/abp_t_$L.log 2>&1; rc=$?
    echo "== $L tests rc=$rc"; grep -E "^prefill|batch-1 decode|batch-16 decode|off the oracle|passed|failed" $O/abp_t_$L.log | cut -c1-220
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  fi
  R=$PWD
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/abp_prof_$L" -o run -- python3 -u "$R/tools/prefill_bench.py" --iters 3) > $O/abp_b_$L.log 2>&1 || exit 1
  echo "== $L bench"; tail -1 $O/abp_b_$L.log | cut -c1-200
  python3 tools/prof_summary.py "$O/abp_prof_$L" > "$O/abp_k_$L.txt" 2>&1 || exit 1
  rm -rf "$O/abp_prof_$L"
  grep -E "attn|pgemm" "$O/abp_k_$L.txt" | head -6 | cut -c1-200
done
