set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_split.so
timeout -k 10 600 $P tests/test_gpu_configs.py -k "attention_kernels or kv_attention_cosine or batch128" > gpurun_out/tsp.log 2>&1; grep -h "passed\|failed\|attention b" gpurun_out/tsp.log | cut -c1-160
timeout -k 10 600 $P tests/test_gpu_reference_golden.py -k "batch128" > gpurun_out/tsp2.log 2>&1; grep -h "passed\|failed\|vs reference" gpurun_out/tsp2.log | cut -c1-200
unset WF_BITNET_LIB
LIBS="libwfbitnet_split.so libwfbitnet.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 10 --no-sub
LIBS="libwfbitnet_split.so libwfbitnet.so" bash tools/ab_bench.sh --batch 128 --steps 30 --warmup 5 --no-sub --ctx-dist uniform
