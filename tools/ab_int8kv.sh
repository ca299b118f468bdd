#!/bin/bash
# int8 K/V batch-128 A/B: the int8 parity tests on the product library, then bench.py --batch 128 --kv int8
# (ctx 1024 and config-4 contexts) alternated with lib/libwfbitnet_$VAR.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -k "int8 or kv" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/i8_tests.log 2>&1 || { tail -30 $O/i8_tests.log; exit 1; }
tail -1 $O/i8_tests.log
for rep in 1 2; do
  for L in product $VAR; do
    if [ $L = product ]; then unset WF_BITNET_LIB; else export WF_BITNET_LIB=$PWD/wrinklefree-inference-engine_amd/lib/libwfbitnet_$L.so; fi
    for D in fixed uniform; do
      timeout -k 10 300 python -u bench.py --batch 128 --kv int8 --ctx-dist $D --steps 50 --warmup 5 --no-cpu-baseline > $O/i8_$L.log 2>&1 || { tail -5 $O/i8_$L.log; exit 1; }
      python3 -c "
import json
d=json.loads([x for x in open('$O/i8_$L.log') if x.startswith('{')][-1])
print('$L $D', d['value'], d['kernels']['attn']['us'], d['roofline']['frac'])"
    done
  done
done
