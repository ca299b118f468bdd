#!/bin/bash
# SQ issue counters of the prefill GEMM kernels per WF_PG_ALG (one --pmc pass each, 8 SQ counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
for a in ${ALGS:-0 3}; do
  rm -rf $R/gpurun_out/pgpmc2/a$a; mkdir -p $R/gpurun_out/pgpmc2
  (cd /tmp && WF_PG_ALG=$a timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv \
      -d $R/gpurun_out/pgpmc2/a$a -o run -- python3 $R/tools/prefill_gemm_bench.py --iters 2 > $R/gpurun_out/pgpmc2/a$a.log 2>&1) || exit 1
  echo "== ALG $a"
  python3 tools/pmc_summary.py gpurun_out/pgpmc2/a$a "k_pgemm_t"
done
