#!/bin/bash
# GPU: optional test subset, then an A/B of the in-tree library against OTHER (if given), then
# the per-phase stamps of render_fwd / field_bwd / tile (scripts/stamps.py) when STAMPS=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi   # (a failed test can be a GPU fault: nothing more runs)
fi
if [ -n "${OTHER:-}" ]; then
  bash scripts/ab_bench.sh "$OTHER" ${ROUNDS:-3} || exit $?
fi
if [ "${STAMPS:-0}" = "1" ]; then
  timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps.log 2>&1
  rc=$?; cat gpurun_out/stamps.log | tail -40; exit $rc
fi
