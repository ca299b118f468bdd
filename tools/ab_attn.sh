# A/B of batched-attention variants (WF_ATTN_VARIANT): parity tests per variant, then batch-128
# bench lines at a fixed context and at config-4 contexts (U[1, 4096), paged)
set -u
for V in 3 4; do
WF_ATTN_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "batched or paged" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_t$V.log 2>&1 || { tail -20 gpurun_out/ab_t$V.log; exit 1; }
echo "V=$V tests: $(tail -1 gpurun_out/ab_t$V.log)"
done
for C in "0 fixed" "3 fixed" "4 fixed" "0 uniform" "3 uniform" "4 uniform"; do
set -- $C
WF_ATTN_VARIANT=$1 timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --ctx-dist $2 > gpurun_out/ab_$1_$2.log 2>&1 || exit 1
echo "V=$1 $2 $(tail -1 gpurun_out/ab_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['us'] for k,v in d['kernels'].items()})")"
done
