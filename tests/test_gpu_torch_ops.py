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


def _channel_major(tm):
    return tm.permute(0, 1, 4, 2, 3)


def _scaled_decoder(inp):
    """EqualizedLinear's gains folded on the host (stylegan.py:173-176), the render_fwd convention."""
    w1, b1, w2, b2 = (inp[k].to(DEV) for k in ('w1', 'b1', 'w2', 'b2'))
    return w1 * (1 / w1.shape[1] ** 0.5), b1, w2 * (1 / w2.shape[1] ** 0.5), b2


def test_render_fwd_bwd_match_volume_render_ops():
    """nfi::render_fwd / render_bwd (channel-major planes, scaled decoder) against
    volume_render_fwd / _bwd on the converted layouts: the same launches, so equal outputs."""
    torch_ops.load()
    inp, planes_tm, dec = _inputs(seed=9, B=2, H=8, S=16)
    cam, focal = inp['cam'].to(DEV), inp['focal'].to(DEV)
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, 8, 8, 1.4)
    pal = inp['palette'].to(DEV)
    planes = inp['planes'].to(DEV)
    rgb, depth, mask, t_sorted, saved = torch.ops.nfi.render_fwd(
        planes, *_scaled_decoder(inp), pal, 1.0, 0.1, ro, rd, near, far, 16, 1.4, False, True, 11, 0)
    ref = torch.ops.nfi.volume_render_fwd(planes_tm, pal, ro, rd, near, far, dec, 16, True, False, True, 1.4, 1.0,
                                          0.1, 0, 11, None, None, True)
    torch.testing.assert_close(rgb, ref[0], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(mask, ref[2], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(t_sorted.reshape(-1, 32), ref[3], rtol=1e-6, atol=1e-7)
    assert t_sorted.shape == (2, 8, 8, 32) and len(saved) == 9
    assert bool((t_sorted[..., 1:] >= t_sorted[..., :-1]).all())
    g = torch.Generator().manual_seed(3)
    g_rgb = torch.randn(2, 8, 8, 3, generator=g).to(DEV)
    g_mask = torch.randn(2, 8, 8, generator=g).to(DEV)
    d_planes, d_pal, d_ro, d_rd = torch.ops.nfi.render_bwd(g_rgb, g_mask, saved, pal, 1.0, 0.1, ro, rd, near, far,
                                                          16, 1.4, False, True)
    rb = torch.ops.nfi.volume_render_bwd(g_rgb.reshape(-1, 3), g_mask.reshape(-1), planes_tm, pal, ro, rd, near,
                                         far, dec, 16, True, False, True, 1.4, 1.0, 0.1, 0, *ref[3:10], True)
    assert d_planes.shape == planes.shape
    assert rel_l2(d_planes, _channel_major(rb[0])) < 1e-5
    assert rel_l2(d_pal, rb[1]) < 1e-5
    assert rel_l2(d_ro, rb[2]) < 1e-5 and rel_l2(d_rd, rb[3]) < 1e-5


def test_composite_ops_match_stages():
    torch_ops.load()
    g = torch.Generator().manual_seed(12)
    sig = (torch.rand(3, 7, 40, generator=g) * 4).to(DEV)
    rgb = torch.rand(3, 7, 40, 3, generator=g).to(DEV)
    rd = torch.nn.functional.normalize(torch.randn(3, 7, 3, generator=g), dim=-1).to(DEV) * 1.3
    t = (torch.sort(torch.rand(3, 7, 40, generator=g), dim=-1)[0] * 2 + 1).to(DEV)
    for white in (False, True):
        out = torch.ops.nfi.composite_fwd(sig, rgb, rd, t, white)
        leaves = [x.clone().requires_grad_() for x in (sig, rgb, rd, t)]
        ref = stages._Composite.apply(*leaves, white, True)
        for a, b in zip(out, ref):
            assert torch.equal(a, b.detach())
        g_rgb = torch.randn(3, 7, 3, generator=g).to(DEV)
        g_mask = torch.randn(3, 7, generator=g).to(DEV)
        g_w = torch.randn(3, 7, 40, generator=g).to(DEV)
        d = torch.ops.nfi.composite_bwd(sig, rgb, rd, t, white, g_rgb, g_mask, g_w)
        torch.autograd.backward([ref[0], ref[2], ref[3]], [g_rgb, g_mask, g_w])
        for a, leaf in zip(d, leaves):
            assert torch.equal(a, leaf.grad)


@pytest.mark.parametrize('heads', [0, 1])
def test_triplane_mlp_ops_match_sampler(heads):
    """triplane_mlp_fwd / _bwd (the sampler closure on world points) against nfi.stages' sampler
    Function on the texel-major planes and the packed decoder."""
    torch_ops.load()
    inp, planes_tm, _ = _inputs(seed=13, B=2, H=8, S=8)
    w1s, b1, w2s, b2 = _scaled_decoder(inp)
    if heads == 1:                                     # RGB_SIGMOID: a 4-row colour head, no palette
        w2s, b2 = w2s[:4].contiguous(), b2[:4].contiguous()
        pal = None
    else:
        pal = inp['palette'].to(DEV)
    dec = ops.pack_decoder(inp['w1'].to(DEV), inp['b1'].to(DEV), inp['w2'].to(DEV)[:w2s.shape[0]],
                           inp['b2'].to(DEV)[:w2s.shape[0]])
    g = torch.Generator().manual_seed(4)
    x = ((torch.rand(2, 300, 3, generator=g) * 2 - 1) * 1.3).to(DEV)
    planes = inp['planes'].to(DEV)
    sigma, rgb, y = torch.ops.nfi.triplane_mlp_fwd(planes, w1s, b1, w2s, b2, pal, x, 1.0, 0.1, 1.4, heads)
    pl = planes_tm.clone().requires_grad_()
    pa = None if pal is None else pal.clone().requires_grad_()
    xx = x.clone().requires_grad_()
    rs, rr, ry = stages._Sampler.apply(pl, pa, xx, dec, heads, 1.4, 1.0, 0.1)
    for a, b in ((sigma, rs), (rgb, rr), (y, ry)):
        torch.testing.assert_close(a, b.detach(), rtol=1e-6, atol=1e-7)
    gs = torch.randn(2, 300, generator=g).to(DEV)
    gr = torch.randn(2, 300, 3, generator=g).to(DEV)
    d_planes, d_pal, d_x = torch.ops.nfi.triplane_mlp_bwd(planes, w1s, b1, w2s, b2, pal, x, 1.0, 0.1, 1.4, heads,
                                                          gs, gr)
    torch.autograd.backward([rs, rr], [gs, gr])
    assert d_planes.shape == planes.shape
    assert rel_l2(d_planes, _channel_major(pl.grad)) < 1e-5
    assert rel_l2(d_x, xx.grad) < 1e-5
    if pal is None:
        assert d_pal.numel() == 0
    else:
        assert rel_l2(d_pal, pa.grad) < 1e-5


@pytest.mark.parametrize('case', ['p3d', 'shapenet'])
def test_dispatcher_ops_match_goldens(case):
    """SURVEY §8(b)'s operators on the reference's own golden vectors, with the
    parity bounds of tests/test_gpu_parity.py::check (fp64 oracle + directly against the golden):
    (1) nfi::rays -> nfi::render_fwd / nfi::render_bwd on the reference layouts (channel-major planes,
    gain-scaled decoder W1s = W1/sqrt(32), W2s = W2/sqrt(64) as EqualizedLinear forms them,
    stylegan.py:173-176), d cam / d focal through nfi::rays' autograd from render_bwd's d ro / d rd;
    (2) the scripted render (TorchScript: nfi::rays + nfi::volume_render with nfi::pack_decoder) with
    the reference's draws.  p3d: random draws, pose gradients; shapenet: deterministic mode, white
    background, pose frozen (force_no_cam_grad)."""
    from golden_io import load
    from gpu_helpers import run_oracle64
    from test_gpu_parity import check
    torch_ops.load()
    d, meta = load(f'render_{case}')
    H, W, S = int(meta['H']), int(meta['W']), int(meta['S'])
    sr, white, rnd = float(meta['scene_range']), bool(meta['white_bg']), bool(meta['randomize'])
    ncg = bool(meta['force_no_cam_grad'])
    inv_alpha, beta = 1.0 / float(d['alpha']), float(d['beta'])
    uc = d['u_coarse'].to(DEV).contiguous() if rnd else None
    uf = d['u_fine'].to(DEV).contiguous() if rnd else None
    g_rgb, g_mask = d['g_rgb'].to(DEV), d['g_mask'].to(DEV)
    ref64 = run_oracle64(d, meta)

    # (1) render_fwd / render_bwd
    w1s, b1, w2s, b2 = _scaled_decoder(d)
    cam = d['cam'].to(DEV).requires_grad_(not ncg)
    focal = d['focal'].to(DEV).requires_grad_(not ncg)
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, H, W, sr)
    pal = d['palette'].to(DEV)
    planes = d['planes'].to(DEV)
    rgb, depth, mask, t_sorted, saved = torch.ops.nfi.render_fwd(
        planes, w1s, b1, w2s, b2, pal, inv_alpha, beta, ro.detach(), rd.detach(), near, far, S, sr, white, rnd, 0, 0,
        uc, uf)
    d_planes, d_pal, d_ro, d_rd = torch.ops.nfi.render_bwd(g_rgb, g_mask, saved, pal, inv_alpha, beta, ro.detach(),
                                                          rd.detach(), near, far, S, sr, white, rnd, True, 0,
                                                          not ncg)
    hip = dict(rgb=rgb.cpu(), depth=depth.cpu(), mask=mask.cpu(), d_planes=d_planes.cpu(), d_palette=d_pal.cpu())
    if not ncg:
        torch.autograd.backward([ro, rd], [d_ro, d_rd])
        hip.update(d_cam=cam.grad.cpu(), d_focal=focal.grad.cpu())
    assert ncg or 'd_cam' in d
    print(f'  render_fwd / render_bwd ({case})')
    check(hip, d, ref64)

    # (2) the scripted render with the reference's draws
    cu = torch.jit.CompilationUnit(torch_ops.render_script_source())
    pl = d['planes'].to(DEV).requires_grad_()
    pa = d['palette'].to(DEV).requires_grad_()
    cam2 = d['cam'].to(DEV).requires_grad_(not ncg)
    focal2 = d['focal'].to(DEV).requires_grad_(not ncg)
    dec = torch.ops.nfi.pack_decoder(*(d[k].to(DEV) for k in ('w1', 'b1', 'w2', 'b2')))
    rgb2, depth2, mask2 = cu.render_rays_u(ops.planes_texel_major(pl), pa, dec, cam2, focal2, H, W, S, sr, inv_alpha,
                                           beta, white, rnd, uc, uf)
    ((rgb2 * g_rgb).sum() + (mask2 * g_mask).sum()).backward()
    hip2 = dict(rgb=rgb2.detach().cpu(), depth=depth2.cpu(), mask=mask2.detach().cpu(), d_planes=pl.grad.cpu(),
                d_palette=pa.grad.cpu())
    if not ncg:
        hip2.update(d_cam=cam2.grad.cpu(), d_focal=focal2.grad.cpu())
    print(f'  scripted render ({case})')
    check(hip2, d, ref64)


@pytest.mark.parametrize('nattn', [1, 5, 9])
def test_render_fwd_attention_counts(nattn):
    """nfi::render_fwd with a decoder of N < 10 attention values ([N+1, 64] output
    layer; palette [B,10,3] whose rows N..9 the head must not reach) equals nfi.render's N-value head
    (render.attention_padded: zero rows + a -1e30 bias on the missing logits) — and so the reference's
    softmax over N logits; a zero-biased padded logit would put exp(-max) of mass on rows N..9."""
    torch_ops.load()
    inp, meta = synthetic_inputs(B=2, H=8, W=8, S=16, R=32, scene_range=1.4, seed=60 + nattn)
    w1s, b1, w2s, b2 = _scaled_decoder(inp)
    w2s, b2 = w2s[:nattn + 1].contiguous(), b2[:nattn + 1].contiguous()
    pal = inp['palette'].to(DEV).clone()
    pal[:, nattn:] = 5.0                              # rows the N-value head must never reach
    cam, focal = inp['cam'].to(DEV), inp['focal'].to(DEV)
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, 8, 8, 1.4)
    uc, uf = inp['u_coarse'].to(DEV).contiguous(), inp['u_fine'].to(DEV).contiguous()
    rgb, depth, mask, _, saved = torch.ops.nfi.render_fwd(inp['planes'].to(DEV), w1s, b1, w2s, b2, pal, 1.0, 0.1,
                                                           ro, rd, near, far, 16, 1.4, False, True, 0, 0, uc, uf)
    g = torch.Generator().manual_seed(1)
    g_rgb = torch.randn(2, 8, 8, 3, generator=g).to(DEV)
    d_planes, d_pal, _, _ = torch.ops.nfi.render_bwd(g_rgb, None, saved, pal, 1.0, 0.1, ro, rd, near, far, 16, 1.4,
                                                     False, True, True, 0, False)
    nfi.configure(scene_range=1.4, white_background=False, fine_sampling=True, use_sdf=True, attention_values=nattn,
                  use_viewdir=False)
    pl = inp['planes'].to(DEV).requires_grad_()
    pa = inp['palette'].to(DEV)[:, :nattn].clone().requires_grad_()
    f = nfi.TriplaneField(planes=pl, palette=pa, w1=inp['w1'].to(DEV), b1=inp['b1'].to(DEV),
                          w2=inp['w2'].to(DEV)[:nattn + 1], b2=inp['b2'].to(DEV)[:nattn + 1], alpha=1.0, beta=0.1,
                          attention_values=nattn)
    rgb2, depth2, mask2, _, _, _ = nfi.render(f, 8, 8, cam, focal, None, None, None, 16, randomize=True,
                                              u_coarse=uc, u_fine=uf)
    (rgb2 * g_rgb).sum().backward()
    nfi.configure(attention_values=10)
    torch.testing.assert_close(rgb, rgb2.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(mask, mask2.detach(), rtol=1e-6, atol=1e-7)
    assert rel_l2(d_planes, pl.grad) < 1e-5
    assert rel_l2(d_pal[:, :nattn], pa.grad) < 1e-5
    assert float(d_pal[:, nattn:].abs().max()) == 0.0


def test_pack_decoder_rejects_ambiguous_rows():
    """nfi::pack_decoder: 11 rows = 10 attention values, 4 = the colour head, 33 = view-direction; any
    other row count needs attention_values (a guessed zero-biased padding would be wrong)."""
    torch_ops.load()
    inp, _, _ = _inputs(seed=3, B=1, H=8, S=8)
    w1, b1 = inp['w1'].to(DEV), inp['b1'].to(DEV)
    w2, b2 = inp['w2'].to(DEV), inp['b2'].to(DEV)
    with pytest.raises(RuntimeError, match='ambiguous'):
        torch.ops.nfi.pack_decoder(w1, b1, w2[:6], b2[:6])
    with pytest.raises(RuntimeError, match='does not match'):
        torch.ops.nfi.pack_decoder(w1, b1, w2[:6], b2[:6], 3)
    a = torch.ops.nfi.pack_decoder(w1, b1, w2[:6], b2[:6], 5)
    b = ops.pack_decoder(w1, b1, torch.cat([w2[:6], w2.new_zeros(5, 64)]), torch.cat([b2[:6], b2.new_full((5,), -1e30)]))
    assert torch.equal(a, b)
