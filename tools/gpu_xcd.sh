set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_configs.py -k "attention_kernels" > gpurun_out/t1.log 2>&1; grep -h "passed\|failed" gpurun_out/t1.log | cut -c1-200
timeout -k 10 200 python -u tools/stamps_graph.py --ctx 1024 --reps 20 > gpurun_out/stamps_b1.txt 2>&1 || exit 1
grep "^attn\|^o_proj\|step_ms" gpurun_out/stamps_b1.txt | cut -c1-300
LIBS="libwfbitnet.so libwfbitnet_noxcd.so" bash tools/ab_bench.sh --steps 50 --warmup 10 --no-sub
