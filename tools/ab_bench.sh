#!/bin/bash
# Same-box A/B of library builds on bench.py lines (alternating, 2 reps):
#   LIBS="libwfbitnet.so libwfbitnet_x.so" bash tools/ab_bench.sh [bench.py args]
# Prints tok/s, ms per step and the per-op live timings of each run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$(pwd)/wrinklefree-inference-engine_amd/lib
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in ${LIBS:-libwfbitnet.so}; do
    WF_BITNET_LIB=$L/$lib timeout -k 10 240 python bench.py --no-cpu-baseline --no-gemv "$@" > gpurun_out/ab/last.log 2>&1 \
      || { tail -20 gpurun_out/ab/last.log; exit 1; }
    echo "$lib rep $rep: $(tail -1 gpurun_out/ab/last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items()})")"
  done
done
