set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd)
mkdir -p gpurun_out/pgpmc
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pgpmc/a -o run -- python3 $R/tools/prefill_gemm_bench.py --iters 2 > $R/gpurun_out/pgpmc/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 --kernel-trace --output-format csv -d $R/gpurun_out/pgpmc/b -o run -- python3 $R/tools/prefill_gemm_bench.py --iters 2 > $R/gpurun_out/pgpmc/b.log 2>&1 || exit 1
find $R/gpurun_out/pgpmc -name "*counter_collection.csv" | head
