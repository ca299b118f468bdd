set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 200 python -u tools/stamps_graph.py --ctx 1024 --reps 20 > gpurun_out/stamps_b1.txt 2>&1 || exit 1
grep "^attn\|o_proj\|step_ms" gpurun_out/stamps_b1.txt | cut -c1-300
timeout -k 10 500 $P tests/test_gpu_configs.py -k "attention_kernels" > gpurun_out/t1.log 2>&1; grep -h "passed\|failed" gpurun_out/t1.log | cut -c1-200
timeout -k 10 600 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-gemv --no-sub > gpurun_out/b1.log 2>&1 || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/b1.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["kernels"]["attn"], d["kernels"]["o_proj"])
PY
