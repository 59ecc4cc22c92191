#!/bin/bash
# One renderer-only bench run; prints value, ms/step and the per-stage launch times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-inversion --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
python -c "
import json
d = json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['stages'].items()})"
