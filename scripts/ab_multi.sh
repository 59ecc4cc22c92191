#!/bin/bash
# A/B of several library builds (GPU box): ROUNDS alternating bench.py runs per library, renderer
# only, printing value and per-stage ms.  Usage: scripts/ab_multi.sh [bench args]; libraries from
# LIBS (space-separated paths; "default" = the in-tree libnfi_hip.so).
set -o pipefail
mkdir -p gpurun_out
show() {
  python - "$1" "$2" <<'PYEOF'
import json, sys
line = [x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d = json.loads(line)
print(f"{sys.argv[1]:24s} {d['value']:9.1f}", {k: v['ms'] for k, v in d['stages'].items()}, flush=True)
PYEOF
}
for i in $(seq "${ROUNDS:-2}"); do
  for lib in ${LIBS:-default}; do
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-inversion --no-configs "$@" > gpurun_out/ab_run.log 2>&1 || exit 1
    else
      NFI_AB_OLDER=1 NFI_LIBRARY=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-inversion --no-configs "$@" > gpurun_out/ab_run.log 2>&1 || exit 1
    fi
    show "$(basename $lib)" gpurun_out/ab_run.log || exit 1
  done
done
