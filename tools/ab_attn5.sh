# A/B of the pair-record attention schedule (variant 5) against the default, bf16 and FP8 K/V
set -u
WF_ATTN_VARIANT=5 WF_ATTN_VARIANT8=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "batched or paged or fp8 or prefill" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab5_t.log 2>&1 || { tail -20 gpurun_out/ab5_t.log; exit 1; }
tail -1 gpurun_out/ab5_t.log
for C in "0 fixed bf16" "5 fixed bf16" "0 uniform bf16" "5 uniform bf16" "0 fixed fp8" "5 fixed fp8" "0 uniform fp8" "5 uniform fp8"; do
set -- $C
WF_ATTN_VARIANT=$1 WF_ATTN_VARIANT8=$1 timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --kv $3 --ctx-dist $2 > gpurun_out/ab5.log 2>&1 || exit 1
echo "V=$1 $2 $3 $(tail -1 gpurun_out/ab5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['attn']['us'])")"
done
