#!/bin/bash
# A/B of environment settings on one library (GPU box): ROUNDS alternating renderer-only bench runs per
# setting in ENVS (space-separated; each a comma-separated list of VAR=value, "-" = none), printing
# value and per-stage ms.  Usage: ENVS="NFI_BWD_SLAB=0 NFI_BWD_SLAB=1" bash scripts/ab_env.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
for i in $(seq "${ROUNDS:-2}"); do
  for e in ${ENVS:--}; do
    envs=(); [ "$e" != "-" ] && IFS=',' read -ra envs <<< "$e"
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-inversion --no-configs "$@" > gpurun_out/ab_env.log 2>&1 || exit 1
    python - "$e" gpurun_out/ab_env.log <<'PYEOF'
import json, sys
line = [x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d = json.loads(line)
print(f"{sys.argv[1]:28s} {d['value']:9.1f}", {k: v['ms'] for k, v in d['stages'].items()}, flush=True)
PYEOF
  done
done
