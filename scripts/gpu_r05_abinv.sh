#!/bin/bash
# Round 5: A/B of the inversion legs in one call — the augmentation grid launch and the one-product
# planes backward on (default) vs off (NFI_AFFINE_GRID_HIP=0 NFI_PLANES_BWD_ONE=0), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
for r in 1 2; do
  for v in on off; do
    if [ $v = on ]; then E=""; else E="NFI_AFFINE_GRID_HIP=0 NFI_PLANES_BWD_ONE=0"; fi
    timeout -k 10 300 env $E python -u bench.py --no-cpu-baseline --no-configs > $O/abinv_${v}_$r.log 2> $O/abinv_${v}_$r.err || exit 3
    python - $O/abinv_${v}_$r.log $v <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]
d = json.loads(l)
print(sys.argv[2], 'value', d['value'], 'vgg', d['inversion']['ms_per_step'], 'l1', d['inversion_l1']['ms_per_step'])
PY
  done
done
