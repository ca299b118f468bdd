# A/B of batched-attention variants (WF_ATTN_VARIANT) and KV plane strides (--max-seq) at batch 128
set -u
for C in "0 4096" "2 4096" "0 1280" "2 1280"; do
set -- $C
WF_ATTN_VARIANT=$1 timeout -k 10 300 python bench.py --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --max-seq $2 > gpurun_out/b128_$1_$2.log 2>&1 || exit 1
echo "V=$1 S=$2 $(tail -1 gpurun_out/b128_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['us'] for k,v in d['kernels'].items()})")"
done
