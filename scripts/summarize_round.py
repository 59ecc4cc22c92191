"""Summarise scripts/profile_round.sh output into profiles/<tag>_summary.md and
profiles/latest_counters.json (per-launch HBM bytes of each nfi kernel, stamped with the render
sources' digest so bench.py uses them only for the kernels they describe).

Per kernel: average duration (kernel trace), HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE;
gfx950's FETCH_SIZE counts half the bytes of wide streaming reads, MI355X_MICROARCH.md §HBM;
Infinity-Cache hits are counted too), and from the SQ / TCC passes:
  MFMA FLOP rate   executed matrix-core FLOP: SQ_INSTS_VALU_MFMA_F32 x 2,048 (v_mfma_f32_16x16x4_f32)
                   + SQ_INSTS_VALU_MFMA_F16 x 16,384 (v_mfma_f32_16x16x32_f16) / duration; the fp32
                   work they carry (the split-f16 decoder runs three f16 products per fp32 product:
                   F16 x 16,384 / 3) against the 157.3 TF fp32 dense peak, the executed f16 rate
                   against the 2.5 PF f16 dense peak
  cycles           GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs): the kernel's active clocks
                   per XCD (2.07 GHz effective for the long kernels); duration x 2.4 GHz without it
  MFMA busy        SQ_VALU_MFMA_BUSY_CYCLES / (1,024 SIMDs x cycles): share of SIMD-cycles the matrix
                   pipe is occupied (a 16x16x4 f32 MFMA holds it 32 cycles)
  VALU / cycle     SQ_INSTS_VALU / (1,024 SIMDs x cycles): VALU instructions issued per SIMD-cycle
  VALU issue       SQ_ACTIVE_INST_VALU x 4 / (1,024 x cycles): share of SIMD-cycles issuing VALU
                   (SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
                   MI355X_MICROARCH.md PMC table)
  waves / SIMD     SQ_WAVE_CYCLES x 4 / (1,024 x cycles): mean resident waves per SIMD
  wait share       SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers);
  issue stall      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (ready but not issued: pipe busy, MFMA RAW)
  L2 hit           TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
import csv
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
config = sys.argv[3] if len(sys.argv) > 3 else 'p3d_fwdbwd'
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 8
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLK = 2.4e9
SIMDS = 1024
CUS = 256
XCDS = 8


def short(n):
    return n.split('(')[0].replace('void ', '').split('<')[0].replace('nfi::', '').strip()


def counters(name):
    p = None
    for dp, _, fs in os.walk(os.path.join(src, name)):
        for f in fs:
            if f.endswith('counter_collection.csv'):
                p = os.path.join(dp, f)
    agg = {}
    if p:
        for r in csv.DictReader(open(p)):
            agg.setdefault(short(r['Kernel_Name']), {}).setdefault(r['Counter_Name'], []).append(
                float(r['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


stats_p = None
for dp, _, fs in os.walk(os.path.join(src, 'trace')):
    for f in fs:
        if f.endswith('kernel_stats.csv'):
            stats_p = os.path.join(dp, f)
stats = list(csv.DictReader(open(stats_p)))
ctr = {}
for name in ('fetch', 'write', 'sqa', 'sqb', 'tcc'):
    for k, cs in counters(name).items():
        ctr.setdefault(k, {}).update(cs)

rows, kern = [], {}
for r in stats:
    k = short(r['Name'])
    if not r['Name'].lstrip('void ').startswith('nfi::'):
        continue
    dur = float(r['AverageNs']) * 1e-9
    c = ctr.get(k, {})
    f, w = c.get('FETCH_SIZE'), c.get('WRITE_SIZE')
    hbm = None if f is None or w is None else 2 * f * 1024 + w * 1024
    cyc = c['GRBM_GUI_ACTIVE'] / XCDS if c.get('GRBM_GUI_ACTIVE') else dur * CLK
    d = {'avg_us': dur * 1e6, 'calls': int(r['Calls'])}
    if c.get('GRBM_GUI_ACTIVE'):
        d['clock_GHz'] = cyc / dur / 1e9
    if hbm is not None:
        d.update(fetch_kib=f, write_kib=w, hbm_bytes_corrected=hbm, hbm_GBps=hbm / dur / 1e9, hbm_frac=hbm / dur / 8e12)
    if 'SQ_INSTS_VALU_MFMA_F32' in c:
        f16 = c.get('SQ_INSTS_VALU_MFMA_F16', 0.0)
        fl = c['SQ_INSTS_VALU_MFMA_F32'] * 2048 + f16 * 16384 / 3   # fp32 work carried
        d.update(mfma_insts=c['SQ_INSTS_VALU_MFMA_F32'] + f16, mfma_TFLOPs=fl / dur / 1e12,
                 mfma_flop_frac=fl / dur / 157.3e12)
        if f16:
            d.update(mfma_f16_exec_TFLOPs=f16 * 16384 / dur / 1e12, mfma_f16_exec_frac=f16 * 16384 / dur / 2500e12)
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
        d['mfma_busy'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * SIMDS)
    if 'SQ_INSTS_VALU' in c:
        d['valu_per_simd_cycle'] = c['SQ_INSTS_VALU'] / (cyc * SIMDS)
    if 'SQ_ACTIVE_INST_VALU' in c:
        d['valu_issue_share'] = 4 * c['SQ_ACTIVE_INST_VALU'] / (cyc * SIMDS)
    if 'SQ_WAVE_CYCLES' in c:
        d['waves_per_simd'] = 4 * c['SQ_WAVE_CYCLES'] / (cyc * SIMDS)
        if 'SQ_WAIT_ANY' in c:
            d['wait_share'] = c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']
        if 'SQ_WAIT_INST_ANY' in c:
            d['issue_stall_share'] = c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']
    if 'TCC_HIT_sum' in c:
        tot = c['TCC_HIT_sum'] + c['TCC_MISS_sum']
        d['l2_hit'] = c['TCC_HIT_sum'] / tot if tot else None
    if 'SQ_LDS_BANK_CONFLICT' in c and c.get('SQ_ACTIVE_INST_LDS'):
        d['lds_conflict_per_active'] = c['SQ_LDS_BANK_CONFLICT'] / c['SQ_ACTIVE_INST_LDS']
    d['raw'] = c
    kern[k] = d


def fmt(v, f='{:.3g}'):
    return '' if v is None else f.format(v)


lines = [f'# rocprofv3 summary — {tag}', '',
         f'`scripts/profile_round.sh` on one MI355X: `rocprofv3 --kernel-trace --stats`, then separate '
         f'`--pmc` passes (FETCH_SIZE; WRITE_SIZE; 8 SQ; 8 SQ + GRBM; TCC hit/miss + GRBM) of '
         f'`python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inversion --no-configs` '
         f'(config {config}, B={batch}).  Derived metrics: see scripts/summarize_round.py.', '',
         '| kernel | calls | avg us | HBM GB/launch | HBM TB/s | HBM frac | MFMA fp32-work TF | of fp32 peak | f16 MFMA exec TF | MFMA busy | '
         'VALU issue | VALU/SIMD/cyc | waves/SIMD | wait share | issue stall | L2 hit | clock GHz |',
         '|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|']
for k, d in sorted(kern.items(), key=lambda kv: -kv[1]['avg_us'] * kv[1]['calls']):
    lines.append(f"| `{k}` | {d['calls']} | {d['avg_us']:.1f} | {fmt(d.get('hbm_bytes_corrected') and d['hbm_bytes_corrected'] / 1e9)} | "
                 f"{fmt(d.get('hbm_GBps') and d['hbm_GBps'] / 1e3)} | {fmt(d.get('hbm_frac'))} | "
                 f"{fmt(d.get('mfma_TFLOPs'))} | {fmt(d.get('mfma_flop_frac'))} | {fmt(d.get('mfma_f16_exec_TFLOPs'))} | {fmt(d.get('mfma_busy'))} | "
                 f"{fmt(d.get('valu_issue_share'))} | {fmt(d.get('valu_per_simd_cycle'))} | {fmt(d.get('waves_per_simd'))} | "
                 f"{fmt(d.get('wait_share'))} | {fmt(d.get('issue_stall_share'))} | {fmt(d.get('l2_hit'))} | "
                 f"{fmt(d.get('clock_GHz'))} |")
lines += ['', '## Raw counters (per launch)', '']
for k, d in kern.items():
    if d['raw']:
        lines.append(f'- `{k}`: ' + ', '.join(f'{c} {v:.4g}' for c, v in sorted(d['raw'].items())))
out = os.path.join(root, 'profiles', f'{tag}_summary.md')
open(out, 'w').write('\n'.join(lines) + '\n')

sys.path.insert(0, os.path.join(root, 'nerf-from-image_amd'))
from nfi.build import source_digest  # noqa: E402
js = {k: {kk: vv for kk, vv in d.items() if kk != 'raw'} for k, d in kern.items() if 'hbm_bytes_corrected' in d}
json.dump({'tag': tag, 'source_digest': source_digest(), 'config': config, 'batch': batch,
           'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 per '
                     'MI355X_MICROARCH.md HBM section; SQ/TCC passes in profiles/' + f'{tag}_summary.md',
           'kernels': js}, open(os.path.join(root, 'profiles', 'latest_counters.json'), 'w'), indent=1)
print(out)
