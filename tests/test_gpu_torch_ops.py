"""The TORCH_LIBRARY(nfi, ...) operators (nfi/libnfi_torch.so) on the GPU: a TorchScript render
(torch.ops.nfi.rays + torch.ops.nfi.volume_render, scripted) against the ctypes path (nfi.ops) on
the same inputs and Philox seed — the same kernels, so outputs bit for bit and gradients equal up
to d planes' float-atomic order — and the seam ops against nfi.stages."""

import pytest
import torch

import nfi
from nfi import ops, stages, torch_ops
from gpu_helpers import rel_l2, synthetic_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _inputs(seed=5, B=2, H=16, S=32):
    inp, meta = synthetic_inputs(B=B, H=H, W=H, S=S, R=32, scene_range=1.4, seed=seed)
    planes_tm = ops.planes_texel_major(inp['planes'].to(DEV)).contiguous()
    dec = ops.pack_decoder(inp['w1'].to(DEV), inp['b1'].to(DEV), inp['w2'].to(DEV), inp['b2'].to(DEV))
    return inp, planes_tm, dec


def test_scripted_render_matches_ctypes_path():
    torch_ops.load()
    inp, planes_tm, dec = _inputs()
    cu = torch.jit.CompilationUnit(torch_ops.render_script_source())
    g = torch.Generator().manual_seed(2)
    H, S = 16, 32
    g_rgb = torch.randn(2, H, H, 3, generator=g).to(DEV)
    g_mask = torch.randn(2, H, H, generator=g).to(DEV)
    res = {}
    for path in ('script', 'ctypes'):
        pl = planes_tm.clone().requires_grad_()
        pal = inp['palette'].to(DEV).clone().requires_grad_()
        cam = inp['cam'].to(DEV).clone().requires_grad_()
        focal = inp['focal'].to(DEV).clone().requires_grad_()
        if path == 'script':
            rgb, depth, mask = cu.render_rays(pl, pal, dec, cam, focal, H, H, S, 1.4, 1.0, 0.1, 77, False)
        else:
            ro, rd, near, far = ops.rays(cam, focal, None, None, H, H, 1.4)
            opts = ops.RenderOptions(samples=S, fine=True, white_background=False, randomize=True, scene_range=1.4,
                                     inv_alpha=1.0, beta=0.1)
            rgb, depth, mask = ops.volume_render(pl, pal, ro, rd, near, far, dec, opts, seed=77)
        ((rgb * g_rgb).sum() + (mask * g_mask).sum()).backward()
        res[path] = dict(rgb=rgb.detach(), depth=depth.detach(), mask=mask.detach(), d_planes=pl.grad,
                         d_palette=pal.grad, d_cam=cam.grad, d_focal=focal.grad)
    a, b = res['script'], res['ctypes']
    for k in ('rgb', 'depth', 'mask', 'd_palette', 'd_cam', 'd_focal'):
        assert torch.equal(a[k], b[k]), k
    assert rel_l2(a['d_planes'], b['d_planes']) < 1e-5


def test_fwd_bwd_ops_match_autograd_op():
    """volume_render_fwd / volume_render_bwd as plain ops give the autograd op's values."""
    torch_ops.load()
    inp, planes_tm, dec = _inputs(seed=6, B=1, H=8, S=16)
    cam, focal = inp['cam'].to(DEV), inp['focal'].to(DEV)
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, 8, 8, 1.4)
    pal = inp['palette'].to(DEV)
    args = (planes_tm, pal, ro, rd, near, far, dec, 16, True, False, True, 1.4, 1.0, 0.1, 0)
    out = torch.ops.nfi.volume_render_fwd(*args, 5, None, None, True)
    pl = planes_tm.clone().requires_grad_()
    rgb, depth, mask = torch.ops.nfi.volume_render(pl, pal, ro, rd, near, far, dec, 16, True, False, True, 1.4,
                                                   1.0, 0.1, 0, 5)
    assert torch.equal(out[0], rgb.detach()) and torch.equal(out[2], mask.detach())
    g_rgb = torch.ones_like(rgb).reshape(-1, 3)
    g_mask = torch.zeros_like(mask).reshape(-1)
    bwd = torch.ops.nfi.volume_render_bwd(g_rgb, g_mask, *args, *out[3:10], False)
    rgb.sum().backward()
    assert rel_l2(bwd[0], pl.grad) < 1e-5


def test_seam_ops_match_stages():
    torch_ops.load()
    g = torch.Generator().manual_seed(8)
    x = (torch.rand(20, 70, generator=g) + 0.2).to(DEV).requires_grad_()
    y = torch.ops.nfi.cumprod_exclusive(x)
    x2 = x.detach().clone().requires_grad_()
    y2 = stages.cumprod_exclusive(x2)
    assert torch.equal(y, y2)
    gy = torch.randn(20, 70, generator=g).to(DEV)
    (y * gy).sum().backward()
    (y2 * gy).sum().backward()
    assert torch.equal(x.grad, x2.grad)
    bins = torch.sort(torch.rand(30, 16, generator=g), dim=-1)[0].to(DEV)
    w = torch.rand(30, 15, generator=g).to(DEV)
    assert torch.equal(torch.ops.nfi.sample_pdf(bins, w, 16, True), stages.sample_pdf(bins, w, 16, True))
    ro = (torch.randn(4, 5, 3, generator=g) * 3).to(DEV)
    rd = torch.nn.functional.normalize(torch.randn(4, 5, 3, generator=g), dim=-1).to(DEV)
    n1, f1 = torch.ops.nfi.compute_near_far_planes(ro, rd, 1.4)
    n2, f2 = stages.compute_near_far_planes(ro, rd, 1.4)
    assert torch.equal(n1, n2) and torch.equal(f1, f2)
    sig = torch.rand(4, 5, 24, generator=g).to(DEV) * 3
    t = torch.sort(torch.rand(4, 5, 24, generator=g), dim=-1)[0].to(DEV) + 1
    assert torch.equal(torch.ops.nfi.render_volume_density_weights_only(sig, ro, rd, t),
                       stages.render_volume_density_weights_only(sig, ro, rd, t))
