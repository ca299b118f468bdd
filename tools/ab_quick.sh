#!/bin/bash
# Same-box A/B of the default batch-1 bench line: product library vs lib/libwfbitnet_$VAR.so, alternated.
#   VAR="name [name2 ...]" [ARGS="bench args"] bash tools/ab_quick.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
ARGS=${ARGS:-"--no-cpu-baseline --no-sub --no-gemv --steps 200 --warmup 10"}
for rep in 1 2; do
  for L in product $VAR; do  # (several variants: space-separated)
    if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
    timeout -k 10 300 python -u bench.py $ARGS > $O/ab_$L.log 2>&1 || { tail -5 $O/ab_$L.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open('$O/ab_$L.log') if x.startswith('{')][-1]); k=d.get('kernels') or {}
print('$L', d['value'], d['ms_per_step'], {n: v['us'] for n, v in k.items()})"
  done
done
