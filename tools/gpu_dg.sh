set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "batch128 or batched or paged" > gpurun_out/tdg.log 2>&1; tail -2 gpurun_out/tdg.log | cut -c1-200
LIBS="libwfbitnet.so libwfbitnet_noxdg.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 10 --no-sub
