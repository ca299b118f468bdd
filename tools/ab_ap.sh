#!/bin/bash
# Batch-1 decode attention block shape (-DWF_AP_THREADS / -DWF_AP_U: 512 threads x 4 keys per lane group, 128 x 16)
set -u
mkdir -p gpurun_out/ab
L=$(pwd)/wrinklefree-inference-engine_amd/lib
for v in ap512 ap128; do
  WF_BITNET_LIB=$L/libwfbitnet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "decode or attention" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/t_$v.log 2>&1 || { tail -30 gpurun_out/ab/t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab/t_$v.log)"
done
LIBS="libwfbitnet.so libwfbitnet_ap512.so libwfbitnet_ap128.so" bash tools/ab_bench.sh --steps 200 --warmup 10 || exit 1
LIBS="libwfbitnet.so libwfbitnet_ap512.so libwfbitnet_ap128.so" bash tools/ab_bench.sh --steps 200 --warmup 10 --ctx 4000 || exit 1
