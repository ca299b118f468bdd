set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_v.so
timeout -k 10 800 $P tests/test_gpu_configs.py -k "prefill_8x2048 or prefill_attention" > gpurun_out/tpfa.log 2>&1; grep -h "passed\|failed\|attention:\|attention on\|layer 1" gpurun_out/tpfa.log | cut -c1-200
timeout -k 10 300 python tools/prefill_bench.py > gpurun_out/pfv.txt 2>&1; grep workload gpurun_out/pfv.txt | cut -c1-150
