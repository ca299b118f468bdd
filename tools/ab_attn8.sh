# A/B of FP8-K/V batched-attention schedules (WF_ATTN_VARIANT8): parity tests, then batch-128 lines
set -u
for V in 2 3 4; do
WF_ATTN_VARIANT8=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fp8" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab8_t$V.log 2>&1 || { tail -20 gpurun_out/ab8_t$V.log; exit 1; }
done
for C in "0 fixed" "2 fixed" "3 fixed" "4 fixed" "0 uniform" "2 uniform" "3 uniform" "4 uniform"; do
set -- $C
WF_ATTN_VARIANT8=$1 timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --kv fp8 --ctx-dist $2 > gpurun_out/ab8.log 2>&1 || exit 1
echo "V=$1 $2 $(tail -1 gpurun_out/ab8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['attn']['us'])")"
done
