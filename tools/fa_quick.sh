#!/bin/bash
# prefill attention iteration: parity tests of the prefill path, end-to-end time, one SQ pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc; mkdir -p $O; rm -f $O/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -k "prefill and not variants" --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 120 python tools/prefill_bench.py | cut -c1-110 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/q -o run -- python3 tools/prefill_bench.py --iters 1 > $O/q.log 2>&1 || { tail -5 $O/q.log; exit 1; }
python3 tools/pmc_summary.py $O/q "${1:-prefill_fa}"
rm -rf $O/q
