#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; any fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-100}
fault() { grep -qiE "memory access fault|illegal (address|instruction)|hipErrorIllegal|core dumped|GPU hang" "$1"; }

timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest -m gpu rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if fault gpurun_out/pytest_gpu.log; then echo "GPU fault in tests: stopping"; exit 5; fi
[ "${ONLY_TESTS:-0}" = "1" ] && exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc

timeout -k 10 600 python bench.py --steps $STEPS --warmup 10 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "== bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc

cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof" -o run -- \
    python "$ROOTDIR/bench.py" --steps $STEPS --warmup 10 --no-cpu-baseline > "$ROOTDIR/gpurun_out/prof.log" 2>&1
rc=$?; echo "== rocprof rc=$rc"; tail -3 "$ROOTDIR/gpurun_out/prof.log"
exit $rc
