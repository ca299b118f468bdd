#!/bin/bash
# Round-end evidence on one MI355X: parity tests, smoke, the batch-1 bench line (with the CPU
# baseline), the batch-128 bench line, rocprofv3 kernel stats of both, the HBM-traffic PMC passes
# of both, and the prefill GEMM bench. Outputs under gpurun_out/round/ (copied into profiles/ by
# hand). Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/round
mkdir -p "$O"
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() { echo "== $1"; }
PART=${PART:-all}
on() { [ "$PART" = all ] || [ "$PART" = "$1" ]; }

if on 1; then
step pytest
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -rf > "$O/pytest_gpu.log" 2>&1 || exit $?
tail -2 "$O/pytest_gpu.log"
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
step bench-b1
timeout -k 10 600 python bench.py --steps 200 --warmup 10 > "$O/bench_b1.log" 2>&1 || exit $?
tail -1 "$O/bench_b1.log" | cut -c1-200
step bench-b128
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline > "$O/bench_b128.log" 2>&1 || exit $?
tail -1 "$O/bench_b128.log" | cut -c1-200
step bench-b128-uniform-paged
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline --ctx-dist uniform > "$O/bench_b128u.log" 2>&1 || exit $?
tail -1 "$O/bench_b128u.log" | cut -c1-200
step bench-b128-fp8
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline --kv fp8 > "$O/bench_b128_fp8.log" 2>&1 || exit $?
tail -1 "$O/bench_b128_fp8.log" | cut -c1-200
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline --kv fp8 --ctx-dist uniform > "$O/bench_b128u_fp8.log" 2>&1 || exit $?
tail -1 "$O/bench_b128u_fp8.log" | cut -c1-200
step bench-b128-int8
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline --kv int8 > "$O/bench_b128_int8.log" 2>&1 || exit $?
tail -1 "$O/bench_b128_int8.log" | cut -c1-200
timeout -k 10 600 python bench.py --batch 128 --steps 100 --warmup 10 --no-cpu-baseline --kv int8 --ctx-dist uniform > "$O/bench_b128u_int8.log" 2>&1 || exit $?
tail -1 "$O/bench_b128u_int8.log" | cut -c1-200
step kv-quality
timeout -k 10 600 python -m pytest tests/test_gpu_configs.py -q -s -p no:cacheprovider -k "kv_attention_cosine" > "$O/kv_quality.log" 2>&1 || exit $?
grep "K/V ctx" "$O/kv_quality.log"
step bench-b1-tq
timeout -k 10 600 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-gemv --wfmt tq > "$O/bench_b1_tq.log" 2>&1 || exit $?
tail -1 "$O/bench_b1_tq.log" | cut -c1-200
fi
if on 2; then
for B in 1 128; do
    step "rocprof b$B"
    cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_b$B" -o run -- \
        python3 "$R/bench.py" --batch $B --steps 100 --warmup 10 --no-cpu-baseline --no-gemv --no-sub > "$O/prof_b$B.log" 2>&1 || exit $?
    cd "$R" && python3 tools/prof_summary.py "$O/prof_b$B" > "$O/kernel_stats_b$B.txt" 2>&1 || exit $?
    rm -rf "$O/prof_b$B"  # raw traces: gpurun_out/ must stay under 64 MiB
    OPS=rocprof_ops; [ $B -gt 1 ] && OPS=rocprof_ops_b$B
    python3 tools/rocprof_ops.py "$O/kernel_stats_b$B.txt" "$TAG" $OPS > /dev/null || exit $?
    cp profiles/$OPS.json profiles/${OPS}_$TAG.json "$O/" || exit $?
    for C in FETCH_SIZE WRITE_SIZE; do
        step "pmc $C b$B"
        cd /tmp && timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/pmc_${C}_b$B" -o run -- \
            python3 "$R/bench.py" --batch $B --steps 20 --warmup 5 --no-cpu-baseline --no-op-timing --no-gemv --no-sub > "$O/pmc_${C}_b$B.log" 2>&1 || exit $?
        cd "$R"
    done
    STEM=pmc_traffic; [ $B -gt 1 ] && STEM=pmc_traffic_b$B
    python3 tools/pmc_traffic.py "$O/pmc_FETCH_SIZE_b$B" "$O/pmc_WRITE_SIZE_b$B" "$TAG" $STEM > /dev/null || exit $?
    cp profiles/$STEM.json "$O/" && rm -rf "$O/pmc_FETCH_SIZE_b$B" "$O/pmc_WRITE_SIZE_b$B"
done
fi
if on 3; then
step gemv
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_gemv" -o run -- python3 "$R/tools/gemv_bench.py" > "$O/prof_gemv.log" 2>&1 || exit $?
cd "$R" && python3 tools/prof_summary.py "$O/prof_gemv" > "$O/kernel_stats_gemv.txt" 2>&1 || exit $?
python3 tools/trace_gaps.py "$O/prof_gemv" k_gemv_rows > "$O/gemv_trace_gaps.txt" 2>&1 || exit $?
rm -rf "$O/prof_gemv"
step gemv-stamps
timeout -k 10 300 python tools/gemv_stamps.py > "$O/gemv_stamps.txt" 2>&1 || exit $?
step stamps-b1
timeout -k 10 300 python tools/stamps_graph.py --ctx 1024 > "$O/stamps_b1.txt" 2>&1 || exit $?
tail -1 "$O/prof_gemv.log" | cut -c1-300
step replicas-same-gpu
timeout -k 10 300 python tools/replica_node.py --replicas 2 --same-gpu --steps 300 > "$O/replicas.log" 2>&1 || exit $?
tail -1 "$O/replicas.log" | cut -c1-300
step prefill
timeout -k 10 300 python tools/prefill_gemm_bench.py > "$O/prefill.log" 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_prefill" -o run -- python3 "$R/tools/prefill_gemm_bench.py" --iters 10 > "$O/prof_prefill.log" 2>&1 || exit $?
cd "$R" && python3 tools/prof_summary.py "$O/prof_prefill" > "$O/kernel_stats_prefill.txt" 2>&1 || exit $?
rm -rf "$O/prof_prefill"
tail -1 "$O/prefill.log"
step prefill-e2e
timeout -k 10 300 python tools/prefill_bench.py > "$O/prefill_e2e.log" 2>&1 || exit $?
timeout -k 10 300 python tools/prefill_bench.py --paged >> "$O/prefill_e2e.log" 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_prefill_e2e" -o run -- python3 "$R/tools/prefill_bench.py" --iters 1 > "$O/prof_prefill_e2e.log" 2>&1 || exit $?
cd "$R" && python3 tools/prof_summary.py "$O/prof_prefill_e2e" > "$O/kernel_stats_prefill_e2e.txt" 2>&1 || exit $?
rm -rf "$O/prof_prefill_e2e"
grep workload "$O/prefill_e2e.log"
fi
echo "== done"
