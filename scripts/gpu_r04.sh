#!/bin/bash
# One GPU call of round 4: optional tests (TESTS), an A/B of library builds (LIBS, ROUNDS; see
# ab_multi.sh), and HBM counter passes (FETCH_SIZE, WRITE_SIZE: separate runs) per library in
# CTR_LIBS ("default" = the in-tree build), summarised per kernel by scripts/ctr_kernels.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q ${PYTEST_X--x} --timeout 300 --timeout-method thread -rf -s > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "^\s+(dist|d_x|d_planes|features|grads|both|cp_|d_cam|d_focal|d_ro|d_rd|weights|dsigma|drd|dt) |FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -60
  if [ $rc -ne 0 ]; then exit $rc; fi   # (a failed test can be a GPU fault: nothing more runs)
fi
if [ -n "${LIBS:-}" ]; then
  bash scripts/ab_multi.sh ${BENCH_ARGS:-} || exit $?
fi
for lib in ${CTR_LIBS:-}; do
  name=$(basename $lib .so)
  out=gpurun_out/ctr_$name
  for pass in FETCH_SIZE WRITE_SIZE; do
    if [ "$lib" = default ]; then envl=""; else envl="NFI_LIBRARY=$lib"; fi
    env $envl timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-include-regex 'nfi::' --output-format csv \
        -d $out/$pass -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-inversion \
        --no-configs ${BENCH_ARGS:-} > $out.$pass.log 2>&1 || { echo "ctr $name $pass failed"; tail -5 $out.$pass.log; exit 1; }
  done
  python scripts/ctr_kernels.py $out $name
done
if [ -n "${DET:-}" ]; then
  timeout -k 10 300 python scripts/determinism_probe.py > gpurun_out/det_r04.log 2>&1 || { echo "determinism probe failed"; tail -5 gpurun_out/det_r04.log; exit 1; }
  cat gpurun_out/det_r04.log | grep -v amdgpu.ids
fi
if [ -n "${FULL_BENCH:-}" ]; then
  timeout -k 10 900 python -u bench.py $FULL_BENCH > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -20 gpurun_out/bench_full.err; exit 1; }
  tail -c 3000 gpurun_out/bench_full.log
fi
