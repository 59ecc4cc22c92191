#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-reps 1} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -5 gpurun_out/bench.log
exit $rc2
