"""Diagnostic: one ray rendered alone (nfi.ops.volume_render with the ray as a leaf) vs the oracle
with the same ray: d ray-origin split by dL/d rgb / dL/d mask, then the per-sample grid gradients
of every (sample, plane) entry (the backward workspace, ops.DEBUG_BACKWARD) against the fp64
oracle's grid_sample gradients.  It located the texel-boundary kink described in
tests/test_gpu_parity.py::test_field_heads_seeded (a fine sample 1e-7 of the span from a texel
column takes the other one-sided x-derivative).  Usage (GPU box): python scripts/diag_ray_grid_grads.py [ray]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'nerf-from-image_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402

import gpu_helpers as gh  # noqa: E402
from nfi import ops  # noqa: E402
from oracle import render_oracle as orc  # noqa: E402

DEV = torch.device('cuda:0')
inp, meta = gh.synthetic_inputs(B=2, H=16, W=16, S=64, R=64, scene_range=1.4, seed=40)
inp['w2'], inp['b2'] = inp['w2'][:4].clone(), inp['b2'][:4].clone()
inp['b2'][0] += 0.97
meta.update(attention_values=0, use_sdf=0)
ref = gh.run_oracle(inp, meta, with_grad=False, return_intermediates=True)['inter']
RAY = int(sys.argv[1]) if len(sys.argv) > 1 else 115
b, pix = RAY // 256, RAY % 256
ro0 = ref['ro'].reshape(-1, 3)[RAY].clone()
rd0 = ref['rd'].reshape(-1, 3)[RAY].clone()
near0 = ref['near'].reshape(-1)[RAY].clone()
far0 = ref['far'].reshape(-1)[RAY].clone()
uc = inp['u_coarse'].reshape(-1, 64)[RAY].clone()
uf = inp['u_fine'].reshape(-1, 64)[RAY].clone()
planes = inp['planes'][b:b + 1]


def oracle(dtype, g_rgb, g_mask, heads_sdf=False):
    fld = orc.Field(planes=planes.to(dtype), w1=inp['w1'].to(dtype), b1=inp['b1'].to(dtype),
                    w2=inp['w2'].to(dtype), b2=inp['b2'].to(dtype), palette=None, alpha=None, beta=None,
                    scene_range=1.4, attention_values=0, use_sdf=False)
    # the ray twice (W = 2): sample_pdf's weights.squeeze() (run.py:271) needs more than one ray
    ro = ro0.to(dtype).view(1, 1, 1, 3).repeat(1, 1, 2, 1).requires_grad_()
    rd = rd0.to(dtype).view(1, 1, 1, 3).repeat(1, 1, 2, 1).requires_grad_()
    gb, nf = orc.get_ray_bundle, orc.compute_near_far_planes
    orc.get_ray_bundle = lambda *a, **k: (ro, rd)
    orc.compute_near_far_planes = lambda *a, **k: (near0.to(dtype).view(1, 1, 1).repeat(1, 1, 2),
                                                   far0.to(dtype).view(1, 1, 1).repeat(1, 1, 2))
    nrm = orc.F.normalize
    orc.F.normalize = lambda x, dim=-1: x
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        rgb, depth, mask = orc.render(fld, 1, 2, None, None, None, None, 64, randomize=True,
                                      u_coarse=uc.to(dtype).view(1, 1, 1, 64).repeat(1, 1, 2, 1),
                                      u_fine=uf.to(dtype).view(1, 64).repeat(2, 1))
        rgb, mask = rgb[:, :, :1], mask[:, :, :1]
    finally:
        orc.get_ray_bundle, orc.compute_near_far_planes, orc.F.normalize = gb, nf, nrm
        torch.set_default_dtype(prev)
    ((rgb * g_rgb.to(dtype)).sum() + (mask * g_mask.to(dtype)).sum()).backward()
    return ro.grad[0, 0, 0].double(), rd.grad[0, 0, 0].double()


def hip(g_rgb, g_mask):
    ptm = ops.planes_texel_major(planes.to(DEV))
    dec = ops.pack_decoder(inp['w1'].to(DEV), inp['b1'].to(DEV), inp['w2'].to(DEV), inp['b2'].to(DEV))
    opts = ops.RenderOptions(samples=64, fine=True, randomize=True, scene_range=1.4, heads=3)
    ro = ro0.to(DEV).view(1, 1, 1, 3).requires_grad_()
    rd = rd0.to(DEV).view(1, 1, 1, 3).requires_grad_()
    rgb, depth, mask = ops.volume_render(ptm, None, ro, rd, near0.to(DEV).view(1, 1, 1), far0.to(DEV).view(1, 1, 1),
                                         dec, opts, u_coarse=uc.to(DEV).view(1, 1, 1, 64), u_fine=uf.to(DEV).view(1, 64))
    ((rgb * g_rgb.to(DEV)).sum() + (mask * g_mask.to(DEV)).sum()).backward()
    return ro.grad.reshape(3).double().cpu(), rd.grad.reshape(3).double().cpu()


for label, g_rgb, g_mask in (('rgb+mask', inp['g_rgb'].reshape(-1, 3)[RAY], inp['g_mask'].reshape(-1)[RAY]),
                             ('rgb only', inp['g_rgb'].reshape(-1, 3)[RAY], torch.zeros(())),
                             ('mask only', torch.zeros(3), inp['g_mask'].reshape(-1)[RAY]),
                             ('rgb x', torch.tensor([1., 0, 0]), torch.zeros(())),
                             ('rgb y', torch.tensor([0., 1, 0]), torch.zeros(())),
                             ('rgb z', torch.tensor([0., 0, 1]), torch.zeros(()))):
    g_rgb = g_rgb.view(1, 1, 1, 3).float()
    g_mask = g_mask.reshape(1, 1, 1).float()
    h = hip(g_rgb, g_mask)
    o32 = oracle(torch.float32, g_rgb, g_mask)
    o64 = oracle(torch.float64, g_rgb, g_mask)
    print(f'{label:9s} d_ro hip-64 {[f"{v:+.2e}" for v in (h[0] - o64[0]).tolist()]} 32-64 '
          f'{[f"{v:+.2e}" for v in (o32[0] - o64[0]).tolist()]} |64| {float(o64[0].norm()):.3e}', flush=True)

# per-sample grid gradients (merged order): HIP workspace dpc vs the fp64 oracle's grid.grad
import torch.nn.functional as F  # noqa: E402
calls = []
_gs = F.grid_sample


def gs_hook(i, grid, **k):
    grid.retain_grad()
    calls.append(grid)
    return _gs(i, grid, **k)


g_rgb = inp['g_rgb'].reshape(-1, 3)[RAY].view(1, 1, 1, 3).float()
g_mask = inp['g_mask'].reshape(-1)[RAY].reshape(1, 1, 1).float()
orc.F.grid_sample = gs_hook
oracle(torch.float64, g_rgb, g_mask)
orc.F.grid_sample = _gs
N = 128
og = torch.zeros(N, 3, 2, dtype=torch.float64)
zc = None
coarse = torch.stack([c.grad[0, :64, 0] for c in calls[:3]], 1)      # [64, 3 planes, 2]
fine = torch.stack([c.grad[0, :64, 0] for c in calls[3:6]], 1)
ops.DEBUG_BACKWARD = {}
dbg = {}
ptm = ops.planes_texel_major(planes.to(DEV))
dec = ops.pack_decoder(inp['w1'].to(DEV), inp['b1'].to(DEV), inp['w2'].to(DEV), inp['b2'].to(DEV))
opts = ops.RenderOptions(samples=64, fine=True, randomize=True, scene_range=1.4, heads=3)
ro = ro0.to(DEV).view(1, 1, 1, 3).requires_grad_()
rd = rd0.to(DEV).view(1, 1, 1, 3).requires_grad_()
rgb, depth, mask = ops.volume_render(ptm, None, ro, rd, near0.to(DEV).view(1, 1, 1), far0.to(DEV).view(1, 1, 1),
                                     dec, opts, u_coarse=uc.to(DEV).view(1, 1, 1, 64), u_fine=uf.to(DEV).view(1, 64),
                                     debug=dbg)
((rgb * g_rgb.to(DEV)).sum() + (mask * g_mask.to(DEV)).sum()).backward()
ws = ops.DEBUG_BACKWARD['workspace']
tail = (N * 24 + 255) // 256 * 256
dpc = ws[-tail:][:N * 24].view(torch.float32).view(N, 3, 2).double().cpu()
t_h = dbg['t_sorted'].cpu().reshape(N)
zc_r = dbg['z_coarse'].cpu().reshape(64)
zf_r = dbg['z_fine'].cpu().reshape(64)
allz = torch.cat([zc_r, zf_r])
allg = torch.cat([coarse, fine])
order = torch.sort(allz, stable=True).indices
og = allg[order]
for j in range(N):
    d = (dpc[j] - og[j]).abs().max()
    if d > 1e-4:
        print(f'sample {j} t {float(t_h[j]):.6f} (coarse/fine idx {int(order[j])}): hip {dpc[j].tolist()} oracle {og[j].tolist()}')
print('max per-entry diff', float((dpc - og).abs().max()))
