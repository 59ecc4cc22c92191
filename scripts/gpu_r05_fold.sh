#!/bin/bash
# Round 5: the folded pose / mapper-norm kernels — their tests, the inversion and producer tests,
# then the bench's inversion legs (before: gpurun_out/r05/bench_r05_v1.log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_pose_mapper.py tests/test_gpu_inversion.py tests/test_gpu_producer_ops.py tests/test_producer.py \
  > $O/fold_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 $O/fold_tests.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-configs > $O/fold_bench.log 2>&1; echo "bench rc=$?"
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r05/fold_bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d.get('ms_per_step'))
for k,v in d.items():
    if 'inv' in k: print(k, v)
PY
