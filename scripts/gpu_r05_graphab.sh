#!/bin/bash
# Round 5: inversion legs eager vs HIP-graph replay (bench.py --inv-graph), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
show() {
python - "$1" "$2" <<'PY'
import json, sys
l=[x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d=json.loads(l)
print(sys.argv[1], 'vgg', d['inversion']['ms_per_step'], 'l1', d['inversion_l1']['ms_per_step'], d['inversion']['step_replay'], flush=True)
PY
}
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/gab_eager.log 2>&1 || exit 3
  show eager $O/gab_eager.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 --inv-graph > $O/gab_graph.log 2>&1 || exit 3
  show graph $O/gab_graph.log
done
