"""Per-phase cycle breakdown of render_fwd / field_bwd (profiling build, -DNFI_STAMPS).

Usage (GPU box):  python scripts/stamps.py [config]
Loads nfi/libnfi_hip_stamps.so (built here by `python nerf-from-image_amd/nfi/build.py --stamps`),
runs the bench step a few times and prints, per phase, the s_memtime cycles summed over waves
divided by the number of waves (the wave's wall time in that phase, other waves interleaved).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['NFI_LIBRARY'] = os.path.join(ROOT, 'nerf-from-image_amd', 'nfi', 'libnfi_hip_stamps.so')
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import _lib  # noqa: E402

FWD = ['setup', 'gather', 'mlp', 'head+save y', 'weights+pdf', 'merge', 'composite+save', 'tile counts', 'sums']
BWD = ['setup', 'gather', 'y+head bwd+palette', 'mlp bwd', 'gfeat write', 'bin append', 'd-coord regather',
       'ray atomics']
TILE = ['row wait + stage', 'entry loop', 'tail (first rows)', 'merge + flush']


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'p3d_fwdbwd'
    cfg = bench.CONFIGS[name]
    dev = torch.device('cuda:0')
    batch = bench.make_inputs(cfg, dev, 0)
    lib = _lib.load()
    lib.nfi_debug_stamps.restype = ctypes.c_int32
    lib.nfi_debug_stamps.argtypes = [ctypes.c_void_p]
    out = (ctypes.c_uint64 * 32)()
    bench.run_step(nfi, batch, cfg, cfg[7])
    torch.cuda.synchronize()
    lib.nfi_debug_stamps(out)
    steps = 3
    for _ in range(steps):
        bench.run_step(nfi, batch, cfg, cfg[7])
    torch.cuda.synchronize()
    assert lib.nfi_debug_stamps(out) == 0
    sr, wbg, flipped, B, H, S, pose, bwd = cfg
    rays = B * H * H
    fwd_waves = rays * steps
    bwd_waves = rays * ((2 * S + 63) // 64) * steps
    print(f'config {name}: {rays} rays; cycles per wave (s_memtime)')
    tot = sum(out[k] for k in range(len(FWD)))
    print('render_fwd (one wave per ray)')
    for k, n in enumerate(FWD):
        print(f'  {n:22s} {out[k] / fwd_waves:10.0f}  {100 * out[k] / max(tot, 1):5.1f}%')
    tot = sum(out[16 + k] for k in range(len(BWD)))
    print('field_bwd (one wave per 64-sample chunk)')
    for k, n in enumerate(BWD):
        print(f'  {n:22s} {out[16 + k] / bwd_waves:10.0f}  {100 * out[16 + k] / max(tot, 1):5.1f}%')
    tot = sum(out[24 + k] for k in range(len(TILE)))
    print('tile chunks (cycles summed over tile waves, per step)')
    for k, n in enumerate(TILE):
        print(f'  {n:22s} {out[24 + k] / steps:14.0f}  {100 * out[24 + k] / max(tot, 1):5.1f}%')


if __name__ == '__main__':
    main()
