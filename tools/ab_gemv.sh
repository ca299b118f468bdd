#!/bin/bash
# Same-box A/B of the standalone bitnet_gemv shapes (tools/gemv_bench.py, graph-replayed per-call
# times): product library vs lib/libwfbitnet_$VAR.so, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
for rep in 1 2; do
  for L in product $VAR; do
    if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
    timeout -k 10 300 python -u tools/gemv_bench.py > $O/gemv_$L.log 2>&1 || { tail -5 $O/gemv_$L.log; exit 1; }
    python3 -c "
import json
d=json.loads([x for x in open('$O/gemv_$L.log') if x.startswith('{')][-1])
print('$L', {k: v.get('us') for k, v in d.items()})"
  done
done
