set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_reference_golden.py -k "prefill" > gpurun_out/tpf.log 2>&1; grep -h "passed\|failed\|vs reference\|vs oracle" gpurun_out/tpf.log | cut -c1-250
bash tools/prof_prefill.sh ${1:-cur}
