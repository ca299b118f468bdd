set -u
mkdir -p gpurun_out/ab
echo "== parity s1x4 (batch<16 decode)"
WF_BITNET_LIB=$(pwd)/wrinklefree-inference-engine_amd/lib/libwfbitnet_s1x4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "decode" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/t_s1x4.log 2>&1; tail -1 gpurun_out/ab/t_s1x4.log
echo "== parity s4 (batch>=16)"
WF_BITNET_LIB=$(pwd)/wrinklefree-inference-engine_amd/lib/libwfbitnet_s4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "batched or paged" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/t_s4.log 2>&1; tail -1 gpurun_out/ab/t_s4.log
echo "== b1"
LIBS="libwfbitnet.so libwfbitnet_s1x4.so" bash tools/ab_bench.sh --steps 200 --warmup 10 || exit 1
echo "== b128 fixed"
LIBS="libwfbitnet.so libwfbitnet_s4.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 || exit 1
echo "== b128 uniform paged"
LIBS="libwfbitnet.so libwfbitnet_s4.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --ctx-dist uniform --paged || exit 1
