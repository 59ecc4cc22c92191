"""Per-step kernel table of an inversion-step trace (scripts/profile_inversion.sh): kernels between
consecutive render_fwd launches (one per step), after the first 4 steps (MIOpen search, warm-up).
Usage: python scripts/inversion_step_table.py gpurun_out/prof_inv_<tag> <tag> [label]
Writes profiles/<tag>_inversion_summary.md."""
import collections
import csv
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
label = sys.argv[3] if len(sys.argv) > 3 else ''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rows = list(csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_trace.csv'))))
rows.sort(key=lambda x: int(x['Start_Timestamp']))
steps = [i for i, x in enumerate(rows) if 'render_fwd' in x['Kernel_Name']]
a, b = steps[4], steps[-1]
n = len(steps) - 1 - 4
win = rows[a:b]


def dur(x):
    return (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e6


def group(name):
    if 'nfi::gemm::' in name:
        return 'GEMMs (nfi split-f16)'
    if 'nfi::syn::lpips' in name:
        return 'LPIPS distance head (nfi HIP)'
    if 'nfi::wino::' in name:
        return 'Winograd transforms (nfi HIP)'
    if 'nfi::dconv::' in name:
        return 'direct convolutions (nfi split-f16)'
    if 'nfi::syn::' in name:
        return 'producer epilogues (nfi HIP)'
    if 'nfi::' in name:
        return 'renderer (nfi HIP)'
    if 'Conv' in name or 'conv' in name or 'igemm' in name:
        return 'convolutions (MIOpen)'
    if name.startswith('Cijk'):
        return 'GEMMs (hipBLASLt/Tensile)'
    if 'at::native' in name:
        return 'PyTorch elementwise/reduce/pool'
    return 'other (transposes, fills, copies)'


span = (int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e6 / n
busy = sum(dur(x) for x in win) / n
by_group = collections.defaultdict(lambda: [0, 0.0])
by_kernel = collections.defaultdict(lambda: [0, 0.0])
for x in win:
    g = group(x['Kernel_Name'])
    by_group[g][0] += 1
    by_group[g][1] += dur(x)
    k = x['Kernel_Name'].split('(')[0][:90]
    by_kernel[k][0] += 1
    by_kernel[k][1] += dur(x)
out = [f'# Inversion step kernels — {tag} {label}', '',
       f'source: `rocprofv3 --kernel-trace --stats` of `scripts/inversion_probe.py` (scripts/profile_inversion.sh); '
       f'{n} steps after 4 warm-up steps.  Span per step {span:.2f} ms (profiled: launch gaps are inflated), '
       f'GPU busy {busy:.2f} ms, {len(win) / n:.0f} kernels per step.', '',
       '| group | kernels/step | ms/step | % of busy |', '|---|---|---|---|']
for g, (c, t) in sorted(by_group.items(), key=lambda kv: -kv[1][1]):
    out.append(f'| {g} | {c / n:.0f} | {t / n:.3f} | {100 * t / n / busy:.1f} |')
out += ['', '| kernel | calls/step | ms/step |', '|---|---|---|']
for k, (c, t) in sorted(by_kernel.items(), key=lambda kv: -kv[1][1])[:25]:
    out.append(f'| `{k}` | {c / n:.1f} | {t / n:.3f} |')
path = os.path.join(root, 'profiles', f'{tag}_inversion_summary.md')
open(path, 'w').write('\n'.join(out) + '\n')
print('\n'.join(out[:14]))
