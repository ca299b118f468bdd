set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 500 $P tests/test_gpu_configs.py -k "attention_kernels" > gpurun_out/t1.log 2>&1; grep -h "attention b\|passed\|failed" gpurun_out/t1.log | cut -c1-400
timeout -k 10 900 $P tests/test_gpu_reference_golden.py -k "batch1 or batch128" > gpurun_out/t3.log 2>&1; grep -h "vs reference\|passed\|failed" gpurun_out/t3.log | cut -c1-600
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-gemv > gpurun_out/b1.log 2>&1 || { echo BFAIL; tail -20 gpurun_out/b1.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --batch 128 --no-cpu-baseline --no-gemv > gpurun_out/b128.log 2>&1 || { echo B128FAIL; tail -20 gpurun_out/b128.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/b1.log", "gpurun_out/b128.log"):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); print(f, d["value"], d["ms_per_step"], json.dumps(d.get("roofline", {}).get("ops", ""))[:600])
PY
