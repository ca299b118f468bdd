#!/bin/bash
# Quick GPU iteration loop: GPU parity tests, then the batch-1 and batch-128 bench lines (no CPU
# baseline). Outputs under gpurun_out/quick/. Every GPU step has its own time limit; the script
# stops at the first failure. Usage: bash tools/quick_gpu.sh [tests|bench|all] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/quick
mkdir -p "$O"
export TMPDIR=/tmp
WHAT=${1:-all}
shift || true
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
    echo "== pytest"
    timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider -rf --timeout 120 \
        --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
    tail -2 "$O/pytest_gpu.log"
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    echo "== bench b1"
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-gemv "$@" > "$O/bench_b1.log" 2>&1 \
        || { tail -20 "$O/bench_b1.log"; exit 1; }
    tail -1 "$O/bench_b1.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items()})"
    echo "== bench b128"
    timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 10 --no-cpu-baseline "$@" > "$O/bench_b128.log" 2>&1 \
        || { tail -20 "$O/bench_b128.log"; exit 1; }
    tail -1 "$O/bench_b128.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items()})"
fi
echo "== done"
