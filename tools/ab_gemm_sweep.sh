#!/bin/bash
# The reference's GEMM batch sweep (bench.gemm_sweep, down projection M 1-32 plus 64) on the product
# library vs lib/libwfbitnet_$VAR.so, alternated twice; then the GEMM / linear parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "gemm or gemv or linear or mlp" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gemm_tests.log 2>&1 || { tail -30 $O/gemm_tests.log; exit 1; }
tail -1 $O/gemm_tests.log
for rep in 1 2; do
  for L in product $VAR; do
    if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
    timeout -k 10 300 python -u -c "
import json, bench
bench.GEMM_SWEEP = (bench.GEMM_SWEEP[0], bench.GEMM_SWEEP[1], (1, 2, 4, 8, 16, 32, 64, 128, 256))
d = bench.gemm_sweep()
print('$L', {m: v['us'] for m, v in d['by_M'].items()})" > $O/sweep_$L.log 2>&1 || { tail -5 $O/sweep_$L.log; exit 1; }
    tail -1 $O/sweep_$L.log
  done
done
