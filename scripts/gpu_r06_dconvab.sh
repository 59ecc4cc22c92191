#!/bin/bash
# Round 6: the inversion legs with the direct convolution (NFI_DCONV=1, default) against the Winograd
# forms (NFI_DCONV=0), two rounds each (bench.py, renderer stages unaffected), then the vgg step's
# kernel trace with the direct convolution.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for i in 1 2; do
  for d in 1 0; do
    NFI_DCONV=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 \
      > $O/dconvab_inv_$d.log 2>&1 || exit 6
    python - $O/dconvab_inv_$d.log dconv=$d <<'PYEOF'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], {k: (d[k]['ms_per_step'], d[k]['rest_ms_per_step']) for k in ('inversion', 'inversion_l1')})
PYEOF
  done
done
TAG=${TAG:-r06d_vgg} LOSS=vgg STEPS=10 bash scripts/profile_inversion.sh || exit 7
echo done
