set -u
mkdir -p gpurun_out/ab
for V in 0 3 4 5; do
  echo "== b128 fixed V=$V";   WF_ATTN_VARIANT=$V bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 || exit 1
  echo "== b128 uniform V=$V"; WF_ATTN_VARIANT=$V bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --ctx-dist uniform --paged || exit 1
done
for V in 0 3 4 5; do
  echo "== fp8 fixed V8=$V";   WF_ATTN_VARIANT8=$V bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --kv fp8 || exit 1
  echo "== fp8 uniform V8=$V"; WF_ATTN_VARIANT8=$V bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --kv fp8 --ctx-dist uniform --paged || exit 1
done
