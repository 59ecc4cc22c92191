#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 0 1 2 4 7; do
  NFI_TILE_DEBUG=$m timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || exit $?
  echo "mode $m: $(tail -1 gpurun_out/abl_$m.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["roofline"]["ms_per_launch"])')"
done
