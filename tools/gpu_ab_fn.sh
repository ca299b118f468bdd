#!/bin/bash
# batch-128 fused row norm study (-DWF_FUSED_NORM, seam words one line each): same-box A/B, then the
# batched parity tests under the study library
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/s2
mkdir -p $O
echo "== ab b128"
LIBS="libwfbitnet.so libwfbitnet_fn.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 10 || exit 1
echo "== tests (fn)"
WF_BITNET_LIB=$(pwd)/wrinklefree-inference-engine_amd/lib/libwfbitnet_fn.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -rf --timeout 180 --timeout-method thread -k "batch128 or batched or paged_kv_equals" > $O/pytest_fn.log 2>&1; tail -3 $O/pytest_fn.log
