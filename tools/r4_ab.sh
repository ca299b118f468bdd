#!/bin/bash
# Round-4 A/B: parity tests on the product library, then same-box bench A/B (batch 1, batch 128)
# of the product library against LIBS' other entries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4ab
mkdir -p "$O"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  eval "timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread -p no:cacheprovider $TESTS" > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
L=$(pwd)/wrinklefree-inference-engine_amd/lib
IFS=';' read -ra BENCHES <<< "${BENCHES:---steps 200 --warmup 20;--batch 128 --steps 50 --warmup 5}"
for args in "${BENCHES[@]}"; do
  for rep in 1 2; do
    for lib in ${LIBS:-libwfbitnet.so}; do
      WF_BITNET_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-gemv $args > "$O/last.log" 2>&1 || { tail -20 "$O/last.log"; exit 1; }
      echo "[$args] $lib rep $rep: $(tail -1 "$O/last.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items()})")"
    done
  done
done
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 300 python tools/stamps_graph.py --ctx 1024 > "$O/stamps_b1.log" 2>&1 || { tail -20 "$O/stamps_b1.log"; exit 1; }
  cat "$O/stamps_b1.log" | cut -c1-600
fi
