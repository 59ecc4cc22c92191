"""The per-stage seams (nfi.stages) against the reference's own stage fixtures
(tests/golden/stages.npz, produced by lib/nerf_utils.py: compute_near_far_planes with cameras
inside the box and rays missing it; sample_pdf deterministic and with injected draws, including
all-zero weights) and against the oracle (fp32 = the reference's op graph, fp64 = truth) with the
bound of tests/test_gpu_parity.py: err(hip, ref64) <= max(FLOOR, K err(ref32, ref64)) and
|hip - ref32| <= FLOOR + K err(ref32, ref64)."""

import pytest
import torch

import nfi
from nfi import stages
from golden_io import load
from gpu_helpers import rel_l2, synthetic_inputs
from oracle import render_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
K = 4.0


def _bound(name, hip, r32, r64, floor, elementwise=False):
    if elementwise:
        def err(a, b):
            return float((a.detach().double().cpu() - b.detach().double().cpu()).abs().max())
    else:
        err = rel_l2
    e_hip, e_ref, e_dir = err(hip, r64), err(r32, r64), err(hip, r32)
    print(f'  {name:10s} hip {e_hip:.3g}  ref32 {e_ref:.3g}  hip-ref32 {e_dir:.3g}')
    assert e_hip <= max(floor, K * e_ref), name
    assert e_dir <= floor + K * e_ref, name


def test_near_far_matches_reference_fixture():
    """nerf_utils.py:227-275 on the fixture's 512 rays (8 cameras inside the box: near clamped to
    0.1; rays missing the box: the hits' min near / max far): bit for bit."""
    d, _ = load('stages')
    near, far = stages.compute_near_far_planes(d['nf_ro'].to(DEV).view(8, 8, 8, 3),
                                               d['nf_rd'].to(DEV).view(8, 8, 8, 3), 1.4)
    assert near.shape == (8, 8, 8)
    assert torch.equal(near.cpu().reshape(-1), d['nf_near'].reshape(-1))
    assert torch.equal(far.cpu().reshape(-1), d['nf_far'].reshape(-1))


def test_sample_pdf_matches_reference_fixture():
    """nerf_utils.py:185-224: deterministic (linspace u) and with the reference's torch.rand draws
    injected; the first 16 rays have all-zero weights (a uniform pdf after + 1e-5).  The weight sum
    is ATen's float sum in its order and the CDF its double-accumulated cumsum, so the bin choice is
    the reference's (at u = 1 too); the interpolation within 1e-5 of each ray's bin span."""
    d, _ = load('stages')
    bins, w = d['pdf_bins'].to(DEV), d['pdf_w'].to(DEV)
    S = bins.shape[-1] + 1
    span = (d['pdf_bins'][:, -1] - d['pdf_bins'][:, 0]).reshape(-1, 1)
    det = stages.sample_pdf(bins, w, S, deterministic=True).cpu()
    rnd = stages.sample_pdf(bins, w, S, deterministic=False, u=d['pdf_u'].to(DEV)).cpu()
    assert float(((det - d['pdf_det']).abs() / span).max()) <= 1e-5
    assert float(((rnd - d['pdf_rnd']).abs() / span).max()) <= 1e-5
    # Philox draws: a valid sample set (inside the bins, deterministic per seed)
    a = stages.sample_pdf(bins, w, S, seed=5)
    b = stages.sample_pdf(bins, w, S, seed=5)
    assert torch.equal(a, b)
    assert bool(((a >= bins[:, :1] - 1e-6) & (a <= bins[:, -1:] + 1e-6)).all())


def _comp_inputs(n=96, N=100, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.sort(torch.rand(n, N, generator=g) * 3 + 1, dim=-1)[0]
    sigma = torch.rand(n, N, generator=g) ** 3 * 8
    rgb = torch.rand(n, N, 3, generator=g) * 2 - 1
    rd = torch.randn(n, 3, generator=g) * 1.3                  # not unit: ||rd|| scales the distances
    ro = torch.randn(n, 3, generator=g)
    normals = torch.nn.functional.normalize(torch.randn(n, N, 3, generator=g), dim=-1)
    sem = torch.softmax(torch.randn(n, N, 10, generator=g), dim=-1)
    gr = [torch.randn(n, 3, generator=g), torch.randn(n, generator=g), torch.randn(n, 3, generator=g),
          torch.randn(n, 10, generator=g)]
    return dict(t=t, sigma=sigma, rgb=rgb, rd=rd, ro=ro, normals=normals, sem=sem), gr


def _comp_run(fn, inp, gr, dtype, dev, white, extras):
    x = {k: v.detach().to(dev, dtype, copy=True).requires_grad_(k in ('t', 'sigma', 'rgb', 'rd', 'normals', 'sem'))
         for k, v in inp.items()}
    out = fn(x['sigma'], x['rgb'], x['ro'], x['rd'], x['t'], normals=x['normals'] if extras else None,
             semantics=x['sem'] if extras else None, white_background=white)
    rgb_map, depth, mask, nmap, smap = out
    loss = (rgb_map * gr[0].to(dev, dtype)).sum() + (mask * gr[1].to(dev, dtype)).sum()
    if extras:
        loss = loss + (nmap * gr[2].to(dev, dtype)).sum() + (smap * gr[3].to(dev, dtype)).sum()
    loss.backward()
    res = {'rgb': rgb_map, 'depth': depth, 'mask': mask}
    if extras:
        res.update(nmap=nmap, smap=smap, d_normals=x['normals'].grad, d_sem=x['sem'].grad)
    res.update(d_sigma=x['sigma'].grad, d_rgb=x['rgb'].grad, d_rd=x['rd'].grad, d_t=x['t'].grad)
    return {k: v.detach().cpu() for k, v in res.items()}


@pytest.mark.parametrize('white,extras,N', [(False, False, 128), (True, False, 100), (True, True, 37),
                                            (False, True, 300)])
def test_render_volume_density(white, extras, N):
    """nerf_utils.py:125-163 with gradients to sigma, rgb, ray_directions (through ||rd||), the
    depth values, and (extras) the normal / semantic maps built on the weights."""
    inp, gr = _comp_inputs(N=N, seed=N)
    hip = _comp_run(stages.render_volume_density, inp, gr, torch.float32, DEV, white, extras)
    r32 = _comp_run(orc.render_volume_density_full, inp, gr, torch.float32, 'cpu', white, extras)
    r64 = _comp_run(orc.render_volume_density_full, inp, gr, torch.float64, 'cpu', white, extras)
    for k in ('rgb', 'mask', 'depth') + (('nmap', 'smap') if extras else ()):
        _bound(k, hip[k], r32[k], r64[k], 2e-5 if k != 'depth' else 1e-4, elementwise=True)
    for k in ('d_sigma', 'd_rgb', 'd_rd', 'd_t') + (('d_normals', 'd_sem') if extras else ()):
        _bound(k, hip[k], r32[k], r64[k], 1e-4)


def _sampler_field(nattn=10, sdf=True, seed=3, B=2, R=32):
    inp, meta = synthetic_inputs(B=B, H=4, W=4, S=8, R=R, scene_range=1.4, seed=seed)
    if nattn == 0:
        inp['w2'], inp['b2'] = inp['w2'][:4].clone(), inp['b2'][:4].clone()
    if not sdf:
        inp['b2'][0] += 0.97
    return inp


def _sampler_run(inp, x, gs, gr, gd, dtype, dev, nattn, sdf, outputs):
    planes = inp['planes'].detach().to(dev, dtype, copy=True).requires_grad_()
    pal = inp['palette'].detach().to(dev, dtype, copy=True).requires_grad_() if nattn else None
    xx = x.detach().to(dev, dtype, copy=True).requires_grad_()
    if dev == DEV:
        nfi.configure(scene_range=1.4)
        f = nfi.TriplaneField(planes=planes, palette=pal, w1=inp['w1'].to(dev), b1=inp['b1'].to(dev),
                              w2=inp['w2'].to(dev), b2=inp['b2'].to(dev), alpha=1.0, beta=0.1,
                              attention_values=nattn, use_sdf=sdf)
        out = stages.make_sampler(f)(xx, outputs)
        sigma, rgb, dist = out['sigma'], out['rgb'], out['sdf_distance']
    else:
        f = orc.Field(planes=planes, w1=inp['w1'].to(dtype), b1=inp['b1'].to(dtype), w2=inp['w2'].to(dtype),
                      b2=inp['b2'].to(dtype), palette=pal, alpha=inp['alpha'].to(dtype), beta=inp['beta'].to(dtype),
                      scene_range=1.4, attention_values=nattn, use_sdf=sdf)
        sigma, rgb, dist = orc.sampler_with_distance(f, xx)
    loss = (sigma * gs.to(dev, dtype)).sum() + (rgb * gr.to(dev, dtype)).sum() + (dist[..., 0] * gd.to(dev, dtype)).sum()
    loss.backward()
    res = {'sigma': sigma, 'rgb': rgb, 'dist': dist[..., 0], 'd_planes': planes.grad, 'd_x': xx.grad}
    if nattn:
        res['d_palette'] = pal.grad
    return {k: v.detach().cpu() for k, v in res.items()}


@pytest.mark.parametrize('nattn,sdf', [(10, True), (0, True), (10, False)])
def test_sampler_closure(nattn, sdf):
    """The sampler closure (generator.py:587-681) at arbitrary points — inside and outside the
    box, on the plane border — forward (sigma, rgb, sdf distance) and backward to the planes, the
    palette and the points (grid_sampler_2d's border / align_corners grid gradient)."""
    inp = _sampler_field(nattn, sdf, seed=7 + nattn + sdf)
    g = torch.Generator().manual_seed(11)
    B, P = 2, 300
    x = (torch.rand(B, P, 3, generator=g) * 2 - 1) * 1.6                # some points outside [-1.4, 1.4]^3
    x[:, :10] = x[:, :10].clamp(-1.4, 1.4)
    gs, gr, gd = torch.randn(B, P, generator=g), torch.randn(B, P, 3, generator=g), torch.randn(B, P, generator=g)
    hip = _sampler_run(inp, x, gs, gr, gd, torch.float32, DEV, nattn, sdf, ('sigma', 'rgb', 'sdf_distance'))
    r32 = _sampler_run(inp, x, gs, gr, gd, torch.float32, 'cpu', nattn, sdf, None)
    r64 = _sampler_run(inp, x, gs, gr, gd, torch.float64, 'cpu', nattn, sdf, None)
    for k in ('sigma', 'rgb', 'dist'):
        _bound(k, hip[k], r32[k], r64[k], 2e-5, elementwise=True)
    for k in ('d_planes', 'd_x') + (('d_palette',) if nattn else ()):
        _bound(k, hip[k], r32[k], r64[k], 1e-3 if k == 'd_planes' else 1e-4)


def test_sampler_extras():
    """'semantics' (softmax of the logits), 'normals' (normalised d distance / d x_in through the
    HIP backward), 'coords' (x_in)."""
    inp = _sampler_field(10, True, seed=21, B=1)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(1, 8, 8, 3, generator=g) * 2 - 1) * 1.2
    nfi.configure(scene_range=1.4)
    f = nfi.TriplaneField(planes=inp['planes'].to(DEV), palette=inp['palette'].to(DEV), w1=inp['w1'].to(DEV),
                          b1=inp['b1'].to(DEV), w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0, beta=0.1)
    out = stages.make_sampler(f)(x.to(DEV), ['normals', 'semantics', 'coords', 'sigma'])
    ref = orc.Field(planes=inp['planes'].double(), w1=inp['w1'].double(), b1=inp['b1'].double(),
                    w2=inp['w2'].double(), b2=inp['b2'].double(), palette=inp['palette'].double(),
                    alpha=inp['alpha'].double(), beta=inp['beta'].double(), scene_range=1.4)
    sigma, rgb, extras = orc.sampler(ref, x.double(), extras=('normals', 'semantics', 'coords'))
    assert out['normals'].shape == x.shape and out['semantics'].shape == (1, 64, 10)
    assert float((out['semantics'].cpu().double() - extras['semantics'].reshape(1, 64, 10)).abs().max()) < 1e-5
    assert float((out['normals'].cpu().double() - extras['normals']).abs().max()) < 1e-4
    assert torch.equal(out['coords'].cpu(), x)
    assert float((out['sigma'].cpu().double() - sigma).abs().max()) < 1e-5


@pytest.mark.parametrize('plane_scale,w_scale,g_scale', [(1.0, 1.0, 1.0), (1e-3, 1.0, 1e-6), (1e3, 1.0, 1e4),
                                                         (1.0, 1e-2, 1.0), (1.0, 30.0, 1e-3)])
def test_decoder_split_precision(plane_scale, w_scale, g_scale):
    """The inversion decoder runs on the f16 matrix cores as hi/lo splits of power-of-two-scaled
    fp32 operands (nfi_render.hip): its outputs and gradients must carry the error
    of an fp32 evaluation at any operand magnitude.  The raw decoder output (sdf distance) and the
    gradients through the decoder backward, with features, weights and loss gradients scaled by
    powers of ten, against the fp64 oracle: err(hip) <= 4 err(fp32 reference) + 1e-6 of the
    value range (no absolute floor)."""
    inp = _sampler_field(10, True, seed=31)
    inp['planes'] = inp['planes'] * plane_scale
    inp['w1'], inp['w2'] = inp['w1'] * w_scale, inp['w2'] * w_scale
    g = torch.Generator().manual_seed(13)
    B, P = 2, 256
    x = (torch.rand(B, P, 3, generator=g) * 2 - 1) * 1.3
    gs, gr, gd = (torch.randn(B, P, generator=g) * g_scale, torch.randn(B, P, 3, generator=g) * g_scale,
                  torch.randn(B, P, generator=g) * g_scale)
    hip = _sampler_run(inp, x, gs, gr, gd, torch.float32, DEV, 10, True, ('sigma', 'rgb', 'sdf_distance'))
    r32 = _sampler_run(inp, x, gs, gr, gd, torch.float32, 'cpu', 10, True, None)
    r64 = _sampler_run(inp, x, gs, gr, gd, torch.float64, 'cpu', 10, True, None)
    d64 = r64['dist'].double()
    e_hip = float((hip['dist'].double() - d64).abs().max())
    e_ref = float((r32['dist'].double() - d64).abs().max())
    print(f'  dist  hip {e_hip:.3g}  ref32 {e_ref:.3g}  (|dist| max {float(d64.abs().max()):.3g})')
    assert e_hip <= 4 * e_ref + 1e-6 * float(d64.abs().max())
    for k in ('d_planes', 'd_x'):
        e_hip, e_ref = rel_l2(hip[k], r64[k]), rel_l2(r32[k], r64[k])
        print(f'  {k:8s} hip {e_hip:.3g}  ref32 {e_ref:.3g}')
        assert e_hip <= 4 * e_ref + 1e-6, k


@pytest.mark.parametrize('spread', ['features', 'grads', 'both'])
def test_decoder_split_wave_spread(spread):
    """Worst case of the per-wave power-of-two scaling of the split-f16 decoder (nfi_render.hip
    split_inputs / the dY scale): inside every 64-point wave ONE point has operands of
    magnitude 1 and the other 63 of magnitude 2^-20 (tap features: the planes are 2^-20 except in the
    region only the outlier samples; and/or loss gradients).  The wave's scale is set by the outlier, so
    a small point's hi/lo pair is exact to 2^-25 of the scaled max, i.e. 2^-(39-k) of its own value at
    2^-k below the max.  Bound: the fp64-relative 4x rule of test_decoder_split_precision over all points
    AND over the small points alone."""
    inp = _sampler_field(10, True, seed=41)
    R = inp['planes'].shape[-1]
    tiny = 2.0 ** -20
    if spread in ('features', 'both'):
        col = torch.arange(R).view(1, 1, 1, 1, R)
        inp['planes'] = torch.where(col >= R // 2 + 2, inp['planes'], inp['planes'] * tiny)
    g = torch.Generator().manual_seed(17)
    B, P = 2, 256
    x = torch.empty(B, P, 3)
    small = torch.ones(B, P, dtype=torch.bool)
    small[:, ::64] = False                                   # the outlier: lane 0 of every wave
    u = torch.rand(B, P, 3, generator=g)
    x[..., :2] = torch.where(small[..., None], -(0.3 + 0.6 * u[..., :2]), 0.3 + 0.6 * u[..., :2]) * 1.4
    x[..., 2] = (u[..., 2] * 2 - 1) * 1.3
    gs, gr, gd = torch.randn(B, P, generator=g), torch.randn(B, P, 3, generator=g), torch.randn(B, P, generator=g)
    if spread in ('grads', 'both'):
        sc = torch.where(small, torch.tensor(tiny), torch.tensor(1.0))
        gs, gr, gd = gs * sc, gr * sc[..., None], gd * sc
    hip = _sampler_run(inp, x, gs, gr, gd, torch.float32, DEV, 10, True, ('sigma', 'rgb', 'sdf_distance'))
    r32 = _sampler_run(inp, x, gs, gr, gd, torch.float32, 'cpu', 10, True, None)
    r64 = _sampler_run(inp, x, gs, gr, gd, torch.float64, 'cpu', 10, True, None)
    for sel, tag in ((torch.ones_like(small), 'all'), (small, 'small')):
        d64 = r64['dist'][sel].double()
        e_hip = float((hip['dist'][sel].double() - d64).abs().max())
        e_ref = float((r32['dist'][sel].double() - d64).abs().max())
        print(f'  {spread:8s} {tag:5s} dist hip {e_hip:.3g} ref32 {e_ref:.3g} (|dist| max {float(d64.abs().max()):.3g})')
        assert e_hip <= 4 * e_ref + 1e-6 * float(d64.abs().max()), (tag, 'dist')
        e_hip, e_ref = rel_l2(hip['d_x'][sel], r64['d_x'][sel]), rel_l2(r32['d_x'][sel], r64['d_x'][sel])
        print(f'  {spread:8s} {tag:5s} d_x  hip {e_hip:.3g} ref32 {e_ref:.3g}')
        assert e_hip <= 4 * e_ref + 1e-6, (tag, 'd_x')
    e_hip, e_ref = rel_l2(hip['d_planes'], r64['d_planes']), rel_l2(r32['d_planes'], r64['d_planes'])
    print(f'  {spread:8s} all   d_planes hip {e_hip:.3g} ref32 {e_ref:.3g}')
    assert e_hip <= 4 * e_ref + 1e-6


@pytest.mark.parametrize('case', ['render_p3d', 'render_shapenet'])
def test_forward_decoder_outputs(case):
    """The decoder inside the fused forward, sample by sample: the decoder outputs the forward saves
    for the backward against an fp64 evaluation of the decoder on the inputs it saved (the golden
    cases' S = 16: 16 of 64 lanes per evaluation, the rest of the wave's tile rows stale — they
    must not enter the per-wave input scale of the split-f16 products)."""
    import torch.nn.functional as F
    from golden_io import load
    d, meta = load(case)
    nfi.configure(scene_range=meta['scene_range'], white_background=bool(meta['white_bg']))
    planes = d['planes'].to(DEV).requires_grad_()
    f = nfi.TriplaneField(planes=planes, palette=d['palette'].to(DEV), w1=d['w1'].to(DEV), b1=d['b1'].to(DEV),
                          w2=d['w2'].to(DEV), b2=d['b2'].to(DEV), alpha=float(d['alpha']), beta=float(d['beta']))
    kw = (dict(randomize=True, u_coarse=d['u_coarse'].to(DEV), u_fine=d['u_fine'].to(DEV)) if meta['randomize']
          else dict(randomize=False))
    rgb = nfi.render(f, meta['H'], meta['W'], d['cam'].to(DEV), d['focal'].to(DEV), None, None, None, meta['S'], **kw)[0]
    fn = rgb.grad_fn
    while fn is not None and len(getattr(fn, 'saved_tensors', ())) < 13:
        fn = fn.next_functions[0][0] if fn.next_functions else None
    st = fn.saved_tensors
    y_saved, x_saved = st[10].cpu().double(), st[12].cpu().double()
    n, nout, N = y_saved.shape
    w1, b1, w2, b2 = (d[k].double() for k in ('w1', 'b1', 'w2', 'b2'))
    y64 = (F.softplus(x_saved @ (w1 / w1.shape[1] ** 0.5).T + b1) @ (w2 / w2.shape[1] ** 0.5).T + b2)
    y64 = y64.view(n, N, nout).transpose(1, 2)
    den = (F.softplus(x_saved @ (w1 / w1.shape[1] ** 0.5).T + b1).abs() @ (w2 / w2.shape[1] ** 0.5).abs().T
           + b2.abs()).view(n, N, nout).transpose(1, 2)
    rel = float(((y_saved - y64).abs() / den).max())
    print(f'  max |y - y64| / sum|terms| = {rel:.3g}')
    assert rel < 2e-6


# ---- the remaining nerf_utils seams (ABI 15), against the reference's own fixture (seams.npz:
# fp32 = the reference functions, fp64 = the same functions on double inputs) -------------------

def _g64(d, key):
    return d[key].double()


def test_seam_cumprod_exclusive():
    """nerf_utils.py:20-25 on rows of 150 (three 64-lane chunks) with exact zeros, a run of ones and a
    zero in the unused last input: forward equal to the reference's fp32 cumprod to one ulp (the fp64
    product is carried in a different association), d x by the 4x rule against fp64."""
    d, _ = load('seams')
    x = d['cp_x'].to(DEV).requires_grad_()
    out = stages.cumprod_exclusive(x)
    (out * d['cp_g'].to(DEV)).sum().backward()
    ref = d['cp_out32']
    ulp = (ref.abs().clamp_min(1e-30) * 2.0 ** -23)
    assert float(((out.detach().cpu() - ref).abs() / ulp).max()) <= 1.0
    assert bool((out[:, 0] == 1).all())
    _bound('cp_out', out.detach().cpu(), ref, _g64(d, 'cp_out64'), 1e-7, elementwise=True)
    _bound('cp_dx', x.grad.cpu(), d['cp_dx32'], _g64(d, 'cp_dx64'), 1e-6)
    assert bool((x.grad[:, -1] == 0).all())


@pytest.mark.parametrize('tag', ['p', 'pcb', 'ob'])
def test_seam_get_ray_bundle(tag):
    """nerf_utils.py:28-93 alone (directions NOT normalised): perspective, perspective + center + bbox,
    ortho + bbox.  Rays bit for bit (ATen's rounding order); d cam / d focal by the 4x rule."""
    d, _ = load('seams')
    B, H, W = 2, 6, 8
    cam = d[f'rb{tag}_cam'].to(DEV).requires_grad_()
    focal = d[f'rb{tag}_focal'].to(DEV).requires_grad_() if f'rb{tag}_focal' in d else None
    center = d[f'rb{tag}_center'].to(DEV) if f'rb{tag}_center' in d else None
    bbox = d[f'rb{tag}_bbox'].to(DEV) if f'rb{tag}_bbox' in d else None
    ro, rd = stages.get_ray_bundle(H, W, focal, cam, bbox, center)
    assert ro.shape == (B, H, W, 3) and rd.shape == (B, H, W, 3)
    assert torch.equal(ro.detach().cpu(), d[f'rb{tag}_ro32'])
    assert torch.equal(rd.detach().cpu(), d[f'rb{tag}_rd32'])
    ((ro * d[f'rb{tag}_gro'].to(DEV)).sum() + (rd * d[f'rb{tag}_grd'].to(DEV)).sum()).backward()
    _bound('d_cam', cam.grad.cpu(), d[f'rb{tag}_dcam32'], _g64(d, f'rb{tag}_dcam64'), 1e-5)
    if focal is not None:
        _bound('d_focal', focal.grad.cpu(), d[f'rb{tag}_dfocal32'], _g64(d, f'rb{tag}_dfocal64'), 1e-5)


@pytest.mark.parametrize('tag', ['d', 'r'])
def test_seam_query_points(tag):
    """nerf_utils.py:96-122: stratified depths and points bit for bit against the reference
    (deterministic, and randomized with its torch.rand_like draws injected); d ro / d rd (the depth
    values carry no gradient) by the 4x rule; a Philox-drawn call reproduces the fused render's coarse
    depths for the same seed."""
    d, _ = load('seams')
    ro, rd = d['qp_ro'].to(DEV).requires_grad_(), d['qp_rd'].to(DEV).requires_grad_()
    near, far = d['qp_near'].to(DEV), d['qp_far'].to(DEV)
    S = d[f'qp{tag}_u'].shape[-1]
    u = d[f'qp{tag}_u'].to(DEV) if tag == 'r' else None
    pts, depth = stages.compute_query_points_from_rays(ro, rd, near, far, S, randomize=(tag == 'r'), u=u)
    assert torch.equal(depth.cpu(), d[f'qp{tag}_depth32'])
    assert torch.equal(pts.detach().cpu(), d[f'qp{tag}_pts32'])
    (pts * d['qp_g'].to(DEV)).sum().backward()
    _bound('d_ro', ro.grad.cpu(), d[f'qp{tag}_dro32'], _g64(d, f'qp{tag}_dro64'), 1e-6)
    _bound('d_rd', rd.grad.cpu(), d[f'qp{tag}_drd32'], _g64(d, f'qp{tag}_drd64'), 1e-6)
    if tag == 'r':
        # Philox: repeatable per seed, inside each stratum
        a = stages.compute_query_points_from_rays(ro.detach(), rd.detach(), near, far, S, seed=11)[1]
        b = stages.compute_query_points_from_rays(ro.detach(), rd.detach(), near, far, S, seed=11)[1]
        assert torch.equal(a, b)
        lo = stages.compute_query_points_from_rays(ro.detach(), rd.detach(), near, far, S, randomize=False)[1]
        step = ((far - near) / S)[..., None]
        assert bool(((a >= lo - 1e-6) & (a <= lo + step * (1 + 1e-5) + 1e-6)).all())


def test_seam_query_points_match_fused_render_draws():
    """The seam's Philox stream is the fused render's coarse stream: same seed, same depths."""
    from gpu_helpers import synthetic_inputs
    inp, meta = synthetic_inputs(B=1, H=8, W=8, S=16, R=16, scene_range=1.4, seed=3)
    nfi.configure(scene_range=1.4)
    f = nfi.TriplaneField(planes=inp['planes'].to(DEV), palette=inp['palette'].to(DEV), w1=inp['w1'].to(DEV),
                          b1=inp['b1'].to(DEV), w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0, beta=0.1)
    dbg = {}
    cam, focal = inp['cam'].to(DEV), inp['focal'].to(DEV)
    with torch.no_grad():
        nfi.render(f, 8, 8, cam, focal, None, None, None, 16, randomize=True, seed=1234, debug=dbg)
        from nfi import ops
        ro, rd, near, far = ops.rays(cam, focal, None, None, 8, 8, 1.4)   # the render's own rays
        depth = stages.compute_query_points_from_rays(ro, rd, near, far, 16, seed=1234)[1]
    assert torch.equal(depth.reshape(-1, 16), dbg['z_coarse'].reshape(-1, 16))


def test_seam_volume_weights():
    """nerf_utils.py:166-182 on rays of 90 samples (empty rays, opaque tails, non-unit directions):
    weights, and the gradients to sigma, the directions (through ||rd||) and the depths, by the
    4x rule against the reference in fp64."""
    d, _ = load('seams')
    sig = d['vw_sigma'].to(DEV).requires_grad_()
    rdw = d['vw_rd'].to(DEV).requires_grad_()
    t = d['vw_t'].to(DEV).requires_grad_()
    w = stages.render_volume_density_weights_only(sig, torch.zeros_like(rdw), rdw, t)
    _bound('weights', w.detach().cpu(), d['vw_w32'], _g64(d, 'vw_w64'), 2e-6, elementwise=True)
    (w * d['vw_g'].to(DEV)).sum().backward()
    for k, x in (('dsigma', sig), ('drd', rdw), ('dt', t)):
        _bound(k, x.grad.cpu(), d[f'vw_{k}32'], _g64(d, f'vw_{k}64'), 1e-5)
