#!/bin/bash
# GPU tests only: TESTS (default: the whole -m gpu suite), no -x; then optionally the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi   # (a failed test can be a GPU fault: no bench after it)
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2> gpurun_out/bench.err
  rc2=$?
  echo "bench rc=$rc2"; tail -5 gpurun_out/bench.err; tail -c 4000 gpurun_out/bench.log
  exit $rc2
fi
exit $rc
