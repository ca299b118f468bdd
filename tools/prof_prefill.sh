#!/bin/bash
# Prefill end-to-end timing (dense + paged) and one rocprofv3 kernel-stats pass of it.
# Outputs under gpurun_out/pf/. Usage: bash tools/prof_prefill.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/pf
mkdir -p "$O"
export TMPDIR=/tmp
TAG=${1:-cur}
timeout -k 10 300 python tools/prefill_bench.py > "$O/prefill_e2e_$TAG.txt" 2>&1 || { tail "$O/prefill_e2e_$TAG.txt"; exit 1; }
timeout -k 10 300 python tools/prefill_bench.py --paged >> "$O/prefill_e2e_$TAG.txt" 2>&1 || { tail "$O/prefill_e2e_$TAG.txt"; exit 1; }
grep workload "$O/prefill_e2e_$TAG.txt"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 "$R/tools/prefill_bench.py" --iters 1 > "$O/prof.log" 2>&1 || { tail "$O/prof.log"; exit 1; }
cd "$R" && python3 tools/prof_summary.py "$O/prof" > "$O/kernel_stats_prefill_e2e_$TAG.txt" 2>&1 || exit 1
rm -rf "$O/prof"
head -14 "$O/kernel_stats_prefill_e2e_$TAG.txt" | cut -c1-150
