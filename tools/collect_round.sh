#!/bin/bash
# Copy the round profile's outputs (gpurun_out/round, tools/profile_round.sh) into profiles/ under
# the round's names:  bash tools/collect_round.sh r04
set -eu
cd "$(dirname "$0")/.."
T=$1; O=gpurun_out/round; P=profiles
last() { tail -1 "$O/$1" > "$P/$2"; }
last bench_b1.log bench_$T.json
last bench_b128.log bench_b128_$T.json
last bench_b128u.log bench_b128_uniform_paged_$T.json
last bench_b128_fp8.log bench_b128_fp8_$T.json
last bench_b128u_fp8.log bench_b128_uniform_paged_fp8_$T.json
last bench_b128_int8.log bench_b128_int8_$T.json
last bench_b128u_int8.log bench_b128_uniform_paged_int8_$T.json
last bench_b1_tq.log bench_tq_$T.json
last replicas.log replicas_same_gpu_$T.json
cp $O/kernel_stats_b1.txt $P/rocprof_${T}_bench_kernel_stats.txt
cp $O/kernel_stats_b128.txt $P/rocprof_${T}_b128_kernel_stats.txt
cp $O/kernel_stats_gemv.txt $P/rocprof_${T}_gemv_kernel_stats.txt
cp $O/kernel_stats_prefill.txt $P/rocprof_${T}_prefill_kernel_stats.txt
cp $O/kernel_stats_prefill_e2e.txt $P/rocprof_${T}_prefill_e2e_kernel_stats.txt
cp $O/pmc_traffic.json $P/pmc_traffic.json; cp $O/pmc_traffic.json $P/pmc_traffic_$T.json
cp $O/pmc_traffic_b128.json $P/pmc_traffic_b128.json; cp $O/pmc_traffic_b128.json $P/pmc_traffic_b128_$T.json
cp $O/rocprof_ops.json $O/rocprof_ops_$T.json $O/rocprof_ops_b128.json $O/rocprof_ops_b128_$T.json $P/
cp $O/gemv_trace_gaps.txt $P/gemv_trace_gaps_$T.txt
grep -v amdgpu.ids $O/gemv_stamps.txt > $P/gemv_stamps_$T.txt
grep -v amdgpu.ids $O/stamps_b1.txt > $P/stamps_b1_$T.txt
grep -v amdgpu.ids $O/prefill.log > $P/prefill_gemm_$T.txt
grep -v amdgpu.ids $O/prefill_e2e.log > $P/prefill_e2e_$T.txt
grep "K/V ctx" $O/kv_quality.log > $P/kv_quality_$T.txt
tail -3 $O/pytest_gpu.log > $P/pytest_gpu_$T.txt
echo "collected $T"
