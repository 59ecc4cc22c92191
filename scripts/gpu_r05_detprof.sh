#!/bin/bash
# Round 5: kernel times of the deterministic mode's backward (sort, tile pass on sorted bins, reduce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/detprof; mkdir -p $O
NFI_DETERMINISTIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --no-cpu-baseline --no-inversion --no-configs --steps 5 --warmup 2 > $O/run.log 2>&1
rc=$?; echo "rc=$rc"
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05/detprof/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, 'us')
PY
