#!/bin/bash
# A/B of an environment switch on the batch-1 bench line: VAR=name VALS="0 1" bash tools/ab_env.sh [bench args]
# (alternating runs, value + per-kernel us)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in ${VALS:-0 1}; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-gemv "$@" \
        > gpurun_out/ab/b_${v}_${rep}.log 2>&1 || { tail -20 gpurun_out/ab/b_${v}_${rep}.log; exit 1; }
    echo -n "$VAR=$v rep $rep: "
    tail -1 gpurun_out/ab/b_${v}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items()})"
  done
done
