#!/bin/bash
# Round 6: batch-1 attention change -- its parity tests, then a same-box A/B against lib/libwfbitnet_base.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_reference_golden.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${PYK:-(step_attention_kernels_vs_oracle and (b1 or untiled)) or timeout or batch1_full or batch1_vs_reference or decode_steps_match or small_batch or graph_equals or decode_attention_vs_oracle}" \
  > $O/attn_tests.log 2>&1 || { tail -40 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
VAR=${VAR:-base} bash tools/ab_quick.sh
