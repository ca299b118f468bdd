#!/bin/bash
# Round-6 GPU checkpoint: parity suite (or a -k selection), smoke, default bench line.
#   PYK="expr" TESTS="tests/..." BENCH=0|1 bash tools/gpu_r06.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 1500 python -u -m pytest $TESTS -m gpu -x -v --timeout 420 --timeout-method thread -p no:cacheprovider -rf ${PYK:+-k "$PYK"} > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
fi
