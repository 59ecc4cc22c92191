#!/bin/bash
# Round 5: the deterministic backward — its tests with the parity, check-build and dispatcher tests,
# then the bench step with NFI_DETERMINISTIC=1 (its cost) and without.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_deterministic.py tests/test_gpu_parity.py tests/test_gpu_tile_check.py tests/test_gpu_torch_ops.py \
  > $O/det_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/det_tests.log
[ $rc -eq 0 ] || exit 3
for det in 0 1; do
  NFI_DETERMINISTIC=$det timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-inversion --no-configs --steps 10 --warmup 3 \
    > $O/det_bench_$det.log 2>&1 || exit 3
  python - "$det" $O/det_bench_$det.log <<'PY'
import json, sys
l=[x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d=json.loads(l)
print('det', sys.argv[1], d['value'], {k: v['ms'] for k, v in d['stages'].items()})
PY
done
