#!/bin/bash
# Batched LM head ring depth (WF_LM_STAGES 3 / 2: two blocks per CU) and 2 attention splits, against the default
set -u
mkdir -p gpurun_out/ab
L=$(pwd)/wrinklefree-inference-engine_amd/lib
for v in lm3 lm2 s2; do
  WF_BITNET_LIB=$L/libwfbitnet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "(batched or paged) and not schedule_variants" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/t_$v.log 2>&1 || { tail -30 gpurun_out/ab/t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab/t_$v.log)"
done
echo "== b128 fixed"
LIBS="libwfbitnet.so libwfbitnet_lm3.so libwfbitnet_lm2.so libwfbitnet_s2.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 || exit 1
echo "== b128 uniform paged"
LIBS="libwfbitnet.so libwfbitnet_s2.so" bash tools/ab_bench.sh --batch 128 --steps 50 --warmup 5 --ctx-dist uniform --paged || exit 1
