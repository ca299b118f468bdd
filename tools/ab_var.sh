#!/bin/bash
# A variant library (lib/libwfbitnet_$VAR.so): its parity tests (-k $PYK), then a same-box A/B of the
# default bench line against the product library (tools/ab_quick.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
if [ -n "${PYK:-}" ]; then
  WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$VAR.so timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py} -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -s -k "$PYK" > $O/var_$VAR.log 2>&1 || { tail -30 $O/var_$VAR.log; exit 1; }
  tail -1 $O/var_$VAR.log
fi
VAR=$VAR bash tools/ab_quick.sh
