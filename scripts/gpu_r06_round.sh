#!/bin/bash
# Round 6 evidence run: the GPU suite, the default bench (driver contract), then the rocprofv3
# passes of the headline config (scripts/profile_round.sh, TAG).  A failed step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_v1}
O=gpurun_out/r06; mkdir -p $O
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider \
    > $O/suite_$TAG.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -15 $O/suite_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench_$TAG.log 2> $O/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -3 $O/bench_$TAG.err; tail -c 3000 $O/bench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  TAG=$TAG bash scripts/profile_round.sh || exit 1
fi
echo done
