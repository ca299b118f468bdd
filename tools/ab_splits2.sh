#!/bin/bash
# Batched decode attention split-count study, round 2 (see DESIGN "Measured negative results"):
# WF_SPLITS=4 / 2 builds against the default 8, bf16 and FP8 K/V, fixed and config-4 contexts.
set -u
mkdir -p gpurun_out/ab
L=$(pwd)/wrinklefree-inference-engine_amd/lib
echo "== full GPU tests with the s4 build"
WF_BITNET_LIB=$L/libwfbitnet_s4.so timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/t_s4_full.log 2>&1 || { tail -30 gpurun_out/ab/t_s4_full.log; exit 1; }
tail -1 gpurun_out/ab/t_s4_full.log
echo "== b128 fixed s4 + DB variant"
WF_ATTN_VARIANT=2 LIBS="libwfbitnet_s4.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 || exit 1
echo "== b128 fixed"
LIBS="libwfbitnet.so libwfbitnet_s4.so libwfbitnet_s2.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 || exit 1
echo "== b128 uniform paged"
LIBS="libwfbitnet.so libwfbitnet_s4.so libwfbitnet_s2.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --ctx-dist uniform --paged || exit 1
echo "== b128 fp8 fixed"
LIBS="libwfbitnet.so libwfbitnet_s4.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --kv fp8 || exit 1
echo "== b128 fp8 uniform paged"
LIBS="libwfbitnet.so libwfbitnet_s4.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --kv fp8 --ctx-dist uniform --paged || exit 1
