#!/bin/bash
# batch-1 iteration: decode parity subset, then same-box A/B of lib/libwfbitnet.so vs libwfbitnet_prev.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/s2
mkdir -p $O
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -rf --timeout 180 --timeout-method thread -k "b1 or decode_steps or graph_equals or batch1 or single or decode_attention" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo "== ab"
LIBS="libwfbitnet.so libwfbitnet_prev.so" bash tools/ab_bench.sh --steps 200 --warmup 10
