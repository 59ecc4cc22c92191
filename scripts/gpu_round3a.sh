#!/bin/bash
# GPU check: full -m gpu suite, a 2-rank gloo rehearsal of bench.py --gpus 2 on the one GPU,
# then the default bench.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NFI_BENCH_DIST=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-configs --inv-steps 3 --inv-loss l1 > gpurun_out/bench_gloo2.log 2>&1
rc2=$?
echo "bench gloo2 rc=$rc2"; tail -c 3000 gpurun_out/bench_gloo2.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 500 python bench.py > gpurun_out/bench.log 2>&1
rc3=$?
echo "bench rc=$rc3"; tail -c 6000 gpurun_out/bench.log
exit $rc3
