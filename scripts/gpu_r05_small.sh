#!/bin/bash
# Round 5: the augmentation grid in one launch (nfi_aug_affine_grid) and the planes layer's backward
# as one product: their tests and the inversion suite, then the default bench (inversion legs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
TAG=${TAG:-small}
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_lpips.py tests/test_gpu_producer_ops.py tests/test_gpu_inversion.py tests/test_gpu_sharded.py \
  > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/${TAG}_bench.log 2> $O/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"
python - <<'PY'
import json, os
t = os.environ.get('TAG', 'small')
l = [x for x in open(f'gpurun_out/r05/{t}_bench.log') if x.startswith('{')][-1]
d = json.loads(l)
print('value', d['value'], 'vgg ms/step', d['inversion']['ms_per_step'], 'l1 ms/step', d['inversion_l1']['ms_per_step'])
PY
