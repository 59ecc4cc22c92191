#!/bin/bash
# Round 5: Winograd image slabs (NFI_WINO_SLAB_MB) — conv tests, then the bench's inversion legs
# with slabs of 128 / 64 MB and without, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_conv.py tests/test_producer.py tests/test_gpu_lpips.py > $O/slab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/slab_tests.log
[ $rc -eq 0 ] || exit 3
show() {
python - "$1" "$2" <<'PY'
import json, sys
l=[x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d=json.loads(l)
print(sys.argv[1], 'vgg', d['inversion']['ms_per_step'], 'l1', d['inversion_l1']['ms_per_step'], flush=True)
PY
}
for r in 1 2; do
  for mb in 128 0 64; do
    NFI_WINO_SLAB_MB=$mb timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/slab_$mb.log 2>&1 || exit 3
    show "slab$mb" $O/slab_$mb.log
  done
done
