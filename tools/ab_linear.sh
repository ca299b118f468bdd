#!/bin/bash
# BitNetLinear at M 16-256 (tools/linear_bench.py) on the product library vs lib/libwfbitnet_$VAR.so,
# after the linear / MLP parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "gemm or gemv or linear or mlp" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/lin_tests.log 2>&1 || { tail -30 $O/lin_tests.log; exit 1; }
tail -1 $O/lin_tests.log
for rep in 1 2; do
  for L in product $VAR; do
    if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
    timeout -k 10 300 python -u tools/linear_bench.py > $O/lin_$L.log 2>&1 || { tail -5 $O/lin_$L.log; exit 1; }
    echo "$L $(tail -1 $O/lin_$L.log)"
  done
done
