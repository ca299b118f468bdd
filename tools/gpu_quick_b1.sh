set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "step_attention_kernels_vs_oracle and (b1 or untiled) or timeout or batch1_full or prefill_attention" > gpurun_out/r06/t3.log 2>&1 || { tail -30 gpurun_out/r06/t3.log; exit 1; }
tail -1 gpurun_out/r06/t3.log
[ -n "${NOSTAMPS:-}" ] || timeout -k 10 300 python -u tools/stamps_graph.py --ctx 1024 > gpurun_out/r06/stamps_b1.txt 2>&1 && python tools/attn_stamps_summary.py >> gpurun_out/r06/stamps_b1.txt || exit 1
grep -A30 "^blocks" gpurun_out/r06/stamps_b1.txt; head -3 gpurun_out/r06/stamps_b1.txt | cut -c1-300
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-sub --no-gemv --steps 100 --warmup 10 > gpurun_out/r06/bench_q.log 2>&1 || exit 1
tail -1 gpurun_out/r06/bench_q.log | cut -c1-200
[ -n "${VAR:-}" ] && { VAR=$VAR bash tools/ab_quick.sh || exit 1; }
