#!/bin/bash
# A/B of the in-tree library against another build (GPU box): alternating bench.py runs, renderer
# only, printing value and per-stage ms of each.  Usage: scripts/ab_bench.sh OTHER.so [rounds] [bench args]
set -o pipefail
other=$1; rounds=${2:-2}; shift 2
mkdir -p gpurun_out
show() {
  python - "$1" "$2" <<'EOF'
import json, sys
line = [x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d = json.loads(line)
print(f"{sys.argv[1]:5s} {d['value']:9.1f}", {k: v['ms'] for k, v in d['stages'].items()}, flush=True)
EOF
}
for i in $(seq "$rounds"); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-inversion --no-configs "$@" > gpurun_out/ab_new.log 2>&1 || exit 1
  show new gpurun_out/ab_new.log || exit 1
  NFI_LIBRARY=$other timeout -k 10 200 python bench.py --no-cpu-baseline --no-inversion --no-configs "$@" > gpurun_out/ab_old.log 2>&1 || exit 1
  show other gpurun_out/ab_old.log || exit 1
done
