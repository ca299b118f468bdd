#!/bin/bash
# A/B of the CPU baseline's GEMV thread-team sizing (oracle/wf_oracle.c, ORC_SIZED_TEAM = one thread per 64 KiB of weights; default every GEMV
# on the whole team), each run a fresh process on the whole CPU share as bench.py's cpu_baseline leg
# runs it; interleaved A B A B. CPU only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
    for v in full sized; do
        D=""; [ $v = sized ] && D="--define ORC_SIZED_TEAM"
        echo "== $v"
        timeout -k 10 120 python -m oracle.cpu_baseline --seconds 5 --gemv-seconds 0.5 $D | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'threads': d['threads'], 'decode': d['decode'], 'gemv': d['gemv']}))" || exit $?
    done
done
