#!/bin/bash
# Round 6: the inversion legs with ENVVAR=1 (default) against ENVVAR=0, ROUNDS alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for i in $(seq ${ROUNDS:-2}); do
  for v in 1 0; do
    env $ENVVAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/envab.log 2>&1 || exit 6
    python - $O/envab.log "$ENVVAR=$v" <<'PYEOF'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], {k: (d[k]['ms_per_step'], d[k]['rest_ms_per_step']) for k in ('inversion', 'inversion_l1')})
PYEOF
  done
done
