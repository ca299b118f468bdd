#!/bin/bash
# SQ counter passes over one prefill (kernel-level breakdown of the prefill attention / GEMMs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
K=${1:-prefill_fa|pgemm_fused<2>}
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/prefill_bench.py --iters 1 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
    python3 tools/pmc_summary.py $O/p$i "$K" >> $O/summary.txt
    rm -rf $O/p$i
done
cat $O/summary.txt
