#!/bin/bash
# Paged-KV check on one MI355X: the paged parity test, then batch-128 lines dense vs paged at a fixed
# context, and the config-4 workload (contexts U[1, max_seq), paged).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "paged or ragged or batched" -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/paged_pytest.log 2>&1 || { tail -30 gpurun_out/paged_pytest.log; exit 1; }
tail -2 gpurun_out/paged_pytest.log
for A in "" "--paged" "--ctx-dist uniform"; do
    timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 5 --no-cpu-baseline $A > gpurun_out/paged_bench.log 2>&1 || { tail -20 gpurun_out/paged_bench.log; exit 1; }
    echo "[$A] $(tail -1 gpurun_out/paged_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('ctx_mean', d['config']['seq_len']), {k:v['us'] for k,v in d['kernels'].items()})")"
done
