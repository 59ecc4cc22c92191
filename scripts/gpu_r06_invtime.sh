#!/bin/bash
# Round 6: GPU tests named in TESTS, then the inversion legs ROUNDS times (bench.py --no-configs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS \
    > $O/invtime_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/invtime_tests.log; [ $rc -eq 0 ] || exit 3
fi
for i in $(seq ${ROUNDS:-2}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/invtime.log 2>&1 || exit 6
  python - $O/invtime.log <<'PYEOF'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(d['value'], {k: (d[k]['ms_per_step'], d[k]['rest_ms_per_step']) for k in ('inversion', 'inversion_l1')})
PYEOF
done
