#!/bin/bash
# Round-4 first GPU check: new parity tests (replicas, reference goldens, K/V codes, attention
# contexts, batched oracle test with its flip report) and a batch-1 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4a
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_replicas.py tests/test_gpu_reference_golden.py \
    "tests/test_gpu_parity.py::test_fp8_kv_codes_and_decode_quality" \
    "tests/test_gpu_configs.py::test_step_attention_kernels_vs_oracle" \
    "tests/test_gpu_configs.py::test_decode_batch128_paged_full_width_vs_oracle" > "$O/pytest.log" 2>&1
rc=$?
tail -15 "$O/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 4 > "$O/bench.log" 2>&1 || exit $?
tail -1 "$O/bench.log" | cut -c1-400
