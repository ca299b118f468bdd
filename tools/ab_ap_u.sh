#!/bin/bash
# batch-1 attention keys per lane group: product (U 10 for one-chunk splits, else 8) vs the previous
# library, at ctx 1024 and 4000, plus the decode parity subset
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_ab_b1.sh || exit 1
echo "== ctx 4000"
LIBS="libwfbitnet.so libwfbitnet_prev.so" bash tools/ab_bench.sh --steps 50 --warmup 10 --ctx 4000 || exit 1
