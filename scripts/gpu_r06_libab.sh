#!/bin/bash
# Round 6: the inversion legs of the in-tree library against an A/B build (LIBB, e.g.
# "libnfi_hip_DNFI_DCONV_STAUX=0.so"), ROUNDS rounds each (bench.py --no-configs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
for i in $(seq ${ROUNDS:-2}); do
  for lib in libnfi_hip.so "$LIBB"; do
    NFI_LIBRARY="$L/$lib" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 \
      > $O/libab.log 2>&1 || exit 6
    python - $O/libab.log "$lib" <<'PYEOF'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], d['value'], {k: (d[k]['ms_per_step'], d[k]['rest_ms_per_step']) for k in ('inversion', 'inversion_l1')})
PYEOF
  done
done
