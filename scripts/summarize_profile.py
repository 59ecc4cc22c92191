"""Summarize a rocprofv3 run (scripts/profile.sh) into profiles/<tag>_summary.md:
per-kernel average duration (kernel trace) and per-launch HBM counters (FETCH_SIZE,
WRITE_SIZE in KiB; gfx950: FETCH_SIZE counts half the bytes of wide streaming reads —
MI355X_MICROARCH.md §HBM — so 'read_bytes_corrected' = 2 x FETCH_SIZE x 1024)."""
import csv
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, 'profiles', f'{tag}_summary.md')
stats = list(csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_stats.csv'))))


def counters(name):
    p = os.path.join(src, name, 'run_counter_collection.csv')
    agg = {}
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            agg.setdefault(r['Kernel_Name'], []).append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch, write = counters('fetch'), counters('write')
lines = [f'# rocprofv3 summary — {tag}', '',
         f'source: `rocprofv3 --kernel-trace --stats` and separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` '
         f'passes of `python3 bench.py` (scripts/profile.sh)', '',
         '| kernel | calls | avg us | % | FETCH_SIZE KiB/launch | read bytes (2x corrected) | WRITE_SIZE KiB/launch |',
         '|---|---|---|---|---|---|---|']
for r in stats:
    n = r['Name']
    short = n.split('(')[0][:70]
    f = fetch.get(n)
    w = write.get(n)
    lines.append(f"| `{short}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.2f} | "
                 f"{'' if f is None else f'{f:.4g}'} | {'' if f is None else f'{2*f*1024/1e9:.3f} GB'} | "
                 f"{'' if w is None else f'{w:.4g}'} |")
open(out, 'w').write('\n'.join(lines) + '\n')
# machine-readable per-launch HBM counters for bench.py's roofline.traffic
import json
kern = {}
for r in stats:
    n = r['Name']
    short = n.split('(')[0].replace('void ', '').split('<')[0].replace('nfi::', '')
    f, w = fetch.get(n), write.get(n)
    if f is None or w is None:
        continue
    kern[short] = {'avg_us': float(r['AverageNs']) / 1e3, 'fetch_kib': f, 'write_kib': w,
                   'hbm_bytes_corrected': 2 * f * 1024 + w * 1024}
sys.path.insert(0, os.path.join(root, 'nerf-from-image_amd'))
from nfi.build import source_digest  # noqa: E402
json.dump({'tag': tag, 'source_digest': source_digest(), 'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), '
           'FETCH_SIZE x2 per MI355X_MICROARCH.md HBM section', 'kernels': kern},
          open(os.path.join(root, 'profiles', 'latest_counters.json'), 'w'), indent=1)
print(out)
