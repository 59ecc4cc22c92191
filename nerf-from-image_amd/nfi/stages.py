"""The reference's per-stage seams as HIP launches (SURVEY §8(b) seams (2) and (3)): a caller that
uses one nerf_utils function, or the Generator's `sampler` closure, without the fused render()
drops these in.  Same names, arguments, shapes and return values as the reference functions;
device tensors only (CPU tensors raise, as everywhere in nfi).

  cumprod_exclusive(tensor)                                            nerf_utils.py:20-25
  get_ray_bundle(height, width, focal_length, tform_cam2world, bbox,
                 center=None)                                          nerf_utils.py:28-93
  compute_query_points_from_rays(ray_origins, ray_directions,
                                 near_thresh, far_thresh, num_samples,
                                 randomize=True)                       nerf_utils.py:96-122
  render_volume_density_weights_only(sigma_a, ray_origins,
                                     ray_directions, depth_values)     nerf_utils.py:166-182
  compute_near_far_planes(ray_origins, ray_directions, scene_range)   nerf_utils.py:227-275
  sample_pdf(bins, weights, num_samples, deterministic=False)          nerf_utils.py:185-224
  render_volume_density(sigma_a, rgb, ray_origins, ray_directions,
                        depth_values, normals=None, semantics=None,
                        white_background=True)                         nerf_utils.py:125-163
  make_sampler(field) / sampler(generator, ws)                         generator.py:587-681

Gradients: render_volume_density / render_volume_density_weights_only to sigma_a, (rgb,)
ray_directions (through ||rd||) and depth_values; cumprod_exclusive to its input; get_ray_bundle to
the camera and the focal length; compute_query_points_from_rays to the rays; the sampler to the
planes, the palette and the points x_in.  near/far and sample_pdf carry none (the reference runs
them under no_grad / on detached inputs).
"""

from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib
from .ops import (HEAD_NERF_DENSITY, HEAD_RGB_SIGMOID, _camera_struct, _ptr, _require_device, _stream, pack_decoder,
                  planes_texel_major)


class _CumprodExclusive(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        lib = _lib.load()
        N = x.shape[-1]
        n = x.numel() // N
        xc = x.contiguous()
        out = torch.empty_like(xc)
        _lib.check(lib.nfi_cumprod_exclusive(_ptr(xc), n, N, _ptr(out), _stream(x.device)), 'nfi_cumprod_exclusive')
        ctx.save_for_backward(xc)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        x, = ctx.saved_tensors
        N = x.shape[-1]
        n = x.numel() // N
        dx = torch.empty_like(x)
        _lib.check(lib.nfi_cumprod_exclusive_backward(_ptr(x), _ptr(g.contiguous()), n, N, _ptr(dx),
                                                      _stream(x.device)), 'nfi_cumprod_exclusive_backward')
        return dx


def cumprod_exclusive(tensor: torch.Tensor) -> torch.Tensor:
    """nerf_utils.py:20-25: the exclusive cumulative product along the last axis (out[..., 0] = 1)."""
    _require_device(tensor)
    if tensor.dtype != torch.float32:
        raise TypeError('nfi: fp32 tensors only')
    if tensor.shape[-1] > 1024 and tensor.requires_grad:
        raise ValueError('cumprod_exclusive backward: at most 1024 entries per row')
    return _CumprodExclusive.apply(tensor)


class _RayBundle(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam, focal, center, bbox, H: int, W: int):
        lib = _lib.load()
        B = cam.shape[0]
        dev = cam.device
        cam_c = cam.contiguous()
        foc_c = None if focal is None else focal.contiguous()
        cen_c = None if center is None else center.contiguous()
        bb_c = None if bbox is None else bbox.contiguous()
        ro = torch.empty((B, H, W, 3), device=dev)
        rd = torch.empty((B, H, W, 3), device=dev)
        cs = _camera_struct(cam_c, foc_c, cen_c, bb_c, H, W)
        _lib.check(lib.nfi_ray_bundle(ctypes.byref(cs), _ptr(ro), _ptr(rd), _stream(dev)), 'nfi_ray_bundle')
        ctx.save_for_backward(cam_c, foc_c, cen_c, bb_c)
        ctx.HW = (H, W)
        return ro, rd

    @staticmethod
    def backward(ctx, g_ro, g_rd):
        lib = _lib.load()
        cam, focal, center, bbox = ctx.saved_tensors
        H, W = ctx.HW
        B = cam.shape[0]
        dev = cam.device
        n = B * H * W
        g_ro = torch.zeros((n, 3), device=dev) if g_ro is None else g_ro.contiguous()
        g_rd = torch.zeros((n, 3), device=dev) if g_rd is None else g_rd.contiguous()
        contrib = torch.empty((n, 16), device=dev)
        cs = _camera_struct(cam, focal, center, bbox, H, W)
        st = _stream(dev)
        _lib.check(lib.nfi_ray_bundle_backward(ctypes.byref(cs), _ptr(g_ro), _ptr(g_rd), _ptr(contrib), st),
                   'nfi_ray_bundle_backward')
        red = torch.empty((B, 16), device=dev)
        ws = torch.empty((B * 64 * 16,), device=dev)
        _lib.check(lib.nfi_segment_sum(_ptr(contrib), B, H * W, 16, _ptr(red), _ptr(ws), st), 'nfi_segment_sum')
        d_cam = torch.zeros((B, 4, 4), device=dev)
        d_cam[:, :3, :] = red[:, :12].view(B, 3, 4)
        d_cam[:, 3, 3] = red[:, 12]
        d_focal = red[:, 13].clone() if focal is not None else None
        return d_cam, d_focal, None, None, None, None


def get_ray_bundle(height: int, width: int, focal_length: Optional[torch.Tensor], tform_cam2world: torch.Tensor,
                   bbox: Optional[torch.Tensor], center: Optional[torch.Tensor] = None):
    """nerf_utils.py:28-93 -> (ray_origins, ray_directions) [B, H, W, 3], the directions NOT
    normalised (perspective when focal_length [B] is given, else orthographic; optional center [B, 2]
    and bbox [B, 2, 2]).  Gradients to tform_cam2world and focal_length (center / bbox: none)."""
    _require_device(tform_cam2world, focal_length, bbox, center)
    if (center is not None and center.requires_grad) or (bbox is not None and bbox.requires_grad):
        raise NotImplementedError('nfi.stages.get_ray_bundle: no gradient to center / bbox')
    return _RayBundle.apply(tform_cam2world, focal_length, center, bbox, int(height), int(width))


class _QueryPoints(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ro, rd, near, far, S: int, randomize: bool, u, seed: int):
        lib = _lib.load()
        lead = ro.shape[:-1]
        n = ro.numel() // 3
        dev = ro.device
        ro_c, rd_c = ro.contiguous(), rd.contiguous()
        nr, fr = near.contiguous(), far.contiguous()
        uu = None if u is None else u.contiguous()
        pts = torch.empty((*lead, S, 3), device=dev)
        depth = torch.empty((*lead, S), device=dev)
        _lib.check(lib.nfi_query_points(_ptr(ro_c), _ptr(rd_c), _ptr(nr), _ptr(fr), n, S, int(randomize), _ptr(uu),
                                        seed & ((1 << 64) - 1), 0, _ptr(pts), _ptr(depth), _stream(dev)),
                   'nfi_query_points')
        ctx.save_for_backward(depth)
        ctx.mark_non_differentiable(depth)
        return pts, depth

    @staticmethod
    def backward(ctx, g_pts, g_depth):
        lib = _lib.load()
        depth, = ctx.saved_tensors
        S = depth.shape[-1]
        n = depth.numel() // S
        dev = depth.device
        lead = depth.shape[:-1]
        d_ro = torch.empty((*lead, 3), device=dev) if ctx.needs_input_grad[0] else None
        d_rd = torch.empty((*lead, 3), device=dev) if ctx.needs_input_grad[1] else None
        if d_ro is None and d_rd is None:
            return None, None, None, None, None, None, None, None
        _lib.check(lib.nfi_query_points_backward(_ptr(depth), _ptr(g_pts.contiguous()), n, S, _ptr(d_ro), _ptr(d_rd),
                                                 _stream(dev)), 'nfi_query_points_backward')
        return d_ro, d_rd, None, None, None, None, None, None


def compute_query_points_from_rays(ray_origins: torch.Tensor, ray_directions: torch.Tensor,
                                   near_thresh: torch.Tensor, far_thresh: torch.Tensor, num_samples: int,
                                   randomize: bool = True, *, u: Optional[torch.Tensor] = None,
                                   seed: Optional[int] = None):
    """nerf_utils.py:96-122 -> (query_points [..., S, 3], depth_values [..., S]) for rays [..., 3] and
    per-ray near / far [...].  randomize: stratified jitter u (far - near) / S with u [..., S] given
    (the reference's torch.rand_like draws) or from a Philox stream (`seed`; with the fused render's
    seed this is the stream its coarse samples draw).  Gradients to the rays (near / far: none)."""
    _require_device(ray_origins, ray_directions, near_thresh, far_thresh, u)
    lead = ray_origins.shape[:-1]
    if (ray_directions.shape != ray_origins.shape or near_thresh.shape != lead or far_thresh.shape != lead
            or ray_origins.shape[-1] != 3):
        raise ValueError('ray_origins / ray_directions [..., 3] and near_thresh / far_thresh [...] expected')
    if near_thresh.requires_grad or far_thresh.requires_grad:
        raise NotImplementedError('nfi.stages.compute_query_points_from_rays: no gradient to near / far '
                                  '(the reference passes detached planes, run.py:197-200)')
    S = int(num_samples)
    if u is not None and u.shape != (*lead, S):
        raise ValueError(f'u must be {(*lead, S)}')
    if seed is None:
        seed = 0 if (not randomize or u is not None) else int(torch.randint(0, 2 ** 62, (1,)).item())
    return _QueryPoints.apply(ray_origins, ray_directions, near_thresh.detach(), far_thresh.detach(), S,
                              bool(randomize), None if u is None else u.detach(), int(seed))


class _VolumeWeights(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigma, rd, t):
        lib = _lib.load()
        N = sigma.shape[-1]
        n = sigma.numel() // N
        dev = sigma.device
        sig_c, rd_c, t_c = sigma.contiguous(), rd.contiguous(), t.contiguous()
        w = torch.empty_like(sig_c)
        _lib.check(lib.nfi_volume_weights_forward(_ptr(sig_c), _ptr(rd_c), _ptr(t_c), n, N, _ptr(w), _stream(dev)),
                   'nfi_volume_weights_forward')
        ctx.save_for_backward(sig_c, rd_c, t_c)
        return w

    @staticmethod
    def backward(ctx, g_w):
        lib = _lib.load()
        sigma, rd, t = ctx.saved_tensors
        N = sigma.shape[-1]
        n = sigma.numel() // N
        dev = sigma.device
        d_sigma = torch.empty_like(sigma)
        d_rd = torch.empty_like(rd) if ctx.needs_input_grad[1] else None
        d_t = torch.empty_like(t) if ctx.needs_input_grad[2] else None
        _lib.check(lib.nfi_volume_weights_backward(_ptr(sigma), _ptr(rd), _ptr(t), n, N, _ptr(g_w.contiguous()),
                                                   _ptr(d_sigma), _ptr(d_rd), _ptr(d_t), _stream(dev)),
                   'nfi_volume_weights_backward')
        return d_sigma, d_rd, d_t


def render_volume_density_weights_only(sigma_a: torch.Tensor, ray_origins: torch.Tensor,
                                       ray_directions: torch.Tensor, depth_values: torch.Tensor) -> torch.Tensor:
    """nerf_utils.py:166-182 -> weights [..., N] = alpha * cumprod_exclusive(1 - alpha + 1e-10) of
    sigma_a [..., N] at depth_values [..., N] (distances scaled by ||ray_directions||; ray_origins is not
    used, as in the reference).  One HIP launch each way (fp64 transmittance scan)."""
    _require_device(sigma_a, ray_directions, depth_values)
    lead = sigma_a.shape[:-1]
    if depth_values.shape != sigma_a.shape or ray_directions.shape != (*lead, 3):
        raise ValueError('sigma_a [..., N], ray_directions [..., 3], depth_values [..., N] expected')
    if sigma_a.shape[-1] > 1024:
        raise ValueError('render_volume_density_weights_only: at most 1024 samples per ray')
    return _VolumeWeights.apply(sigma_a, ray_directions, depth_values)


def compute_near_far_planes(ray_origins: torch.Tensor, ray_directions: torch.Tensor, scene_range: float):
    """nerf_utils.py:227-275 -> (near, far) of shape ray_origins.shape[:-1] (no gradient)."""
    _require_device(ray_origins, ray_directions)
    shape = ray_origins.shape[:-1]
    ro = ray_origins.detach().reshape(-1, 3).contiguous()
    rd = ray_directions.detach().reshape(-1, 3).contiguous()
    n = ro.shape[0]
    lib = _lib.load()
    near = torch.empty(n, device=ro.device)
    far = torch.empty(n, device=ro.device)
    ws = torch.empty(max(1, int(lib.nfi_near_far_workspace_bytes(n))), device=ro.device, dtype=torch.uint8)
    _lib.check(lib.nfi_near_far(_ptr(ro), _ptr(rd), n, float(scene_range), _ptr(near), _ptr(far), _ptr(ws),
                                _stream(ro.device)), 'nfi_near_far')
    return near.view(shape), far.view(shape)


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, num_samples: int, deterministic: bool = False, *,
               u: Optional[torch.Tensor] = None, seed: Optional[int] = None) -> torch.Tensor:
    """nerf_utils.py:185-224: bins [rays, nb], weights [rays, nb-1] -> samples [rays, num_samples]
    (no gradient).  `u` [rays, num_samples] injects the reference's torch.rand draws; otherwise the
    random draws come from a Philox stream (`seed`, or one drawn from torch's CPU generator)."""
    _require_device(bins, weights, u)
    if bins.dim() != 2 or weights.shape != (bins.shape[0], bins.shape[1] - 1):
        raise ValueError(f'bins [rays, nb] and weights [rays, nb-1] expected, got {tuple(bins.shape)} / '
                         f'{tuple(weights.shape)}')
    n, nb = bins.shape
    if u is not None and u.shape != (n, num_samples):
        raise ValueError(f'u must be [{n}, {num_samples}]')
    if seed is None:
        seed = 0 if deterministic or u is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
    out = torch.empty((n, num_samples), device=bins.device)
    b = bins.detach().contiguous()
    w = weights.detach().contiguous()
    uu = None if u is None else u.detach().contiguous()
    lib = _lib.load()
    _lib.check(lib.nfi_sample_pdf(_ptr(b), _ptr(w), n, nb, int(num_samples), int(bool(deterministic)), _ptr(uu),
                                  seed & ((1 << 64) - 1), 0, _ptr(out), _stream(bins.device)), 'nfi_sample_pdf')
    return out


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigma, rgb, rd, t, white: bool, want_w: bool):
        lib = _lib.load()
        N = sigma.shape[-1]
        n = sigma.numel() // N
        dev = sigma.device
        sig_c, rgb_c = sigma.contiguous(), rgb.contiguous()
        rd_c, t_c = rd.contiguous(), t.contiguous()
        rgb_map = torch.empty((n, 3), device=dev)
        depth = torch.empty(n, device=dev)
        mask = torch.empty(n, device=dev)
        w = torch.empty((n, N), device=dev) if want_w else None
        _lib.check(lib.nfi_composite_forward(_ptr(sig_c), _ptr(rgb_c), _ptr(rd_c), _ptr(t_c), n, N, int(white),
                                             _ptr(rgb_map), _ptr(depth), _ptr(mask), _ptr(w), _stream(dev)),
                   'nfi_composite_forward')
        ctx.save_for_backward(sig_c, rgb_c, rd_c, t_c)
        ctx.white, ctx.nN = white, (n, N)
        ctx.mark_non_differentiable(depth)
        lead = sigma.shape[:-1]
        return (rgb_map.view(*lead, 3), depth.view(lead), mask.view(lead),
                w.view(sigma.shape) if w is not None else None)

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_mask, g_w):
        lib = _lib.load()
        sigma, rgb, rd, t = ctx.saved_tensors
        n, N = ctx.nN
        dev = sigma.device
        g_rgb = torch.zeros((n, 3), device=dev) if g_rgb is None else g_rgb.contiguous()
        g_mask = torch.zeros(n, device=dev) if g_mask is None else g_mask.contiguous()
        g_w = None if g_w is None else g_w.contiguous()
        d_sigma = torch.empty_like(sigma)
        d_rgb = torch.empty_like(rgb)
        d_rd = torch.empty_like(rd) if ctx.needs_input_grad[2] else None
        d_t = torch.empty_like(t) if ctx.needs_input_grad[3] else None
        _lib.check(lib.nfi_composite_backward(_ptr(sigma), _ptr(rgb), _ptr(rd), _ptr(t), n, N, int(ctx.white),
                                              _ptr(g_rgb), _ptr(g_mask), _ptr(g_w), _ptr(d_sigma), _ptr(d_rgb),
                                              _ptr(d_rd), _ptr(d_t), _stream(dev)), 'nfi_composite_backward')
        return d_sigma, d_rgb, d_rd, d_t, None, None


def render_volume_density(sigma_a: torch.Tensor, rgb: torch.Tensor, ray_origins: torch.Tensor,
                          ray_directions: torch.Tensor, depth_values: torch.Tensor,
                          normals: Optional[torch.Tensor] = None, semantics: Optional[torch.Tensor] = None,
                          white_background: bool = True):
    """nerf_utils.py:125-163 -> (rgb_map, depth_map, mask, normal_map, semantic_map).  sigma_a
    [..., N], rgb [..., N, 3], ray_directions [..., 3], depth_values [..., N]; the compositing runs
    in one HIP launch each way (fp64 transmittance scan); the normal / semantic maps are formed on
    its weights (normals with the weights detached, as the reference)."""
    _require_device(sigma_a, rgb, ray_origins, ray_directions, depth_values, normals, semantics)
    N = sigma_a.shape[-1]
    lead = sigma_a.shape[:-1]
    if rgb.shape != (*lead, N, 3) or depth_values.shape != sigma_a.shape or ray_directions.shape != (*lead, 3):
        raise ValueError('sigma_a [..., N], rgb [..., N, 3], ray_directions [..., 3], depth_values [..., N] expected')
    want_w = normals is not None or semantics is not None
    rgb_map, depth_map, mask, w = _Composite.apply(sigma_a, rgb, ray_directions, depth_values,
                                                   bool(white_background), want_w)
    normal_map = semantic_map = None
    if normals is not None:
        normal_map = (w[..., None].detach() * normals).sum(dim=-2)
    if semantics is not None:
        semantic_map = (w[..., None] * semantics).sum(dim=-2)
    if white_background and normal_map is not None:
        normal_map = normal_map + (1. - mask[..., None])
    return rgb_map, depth_map, mask, normal_map, semantic_map


# ---------------------------------------------------------------------------------------------
# The sampler closure (generator.py:587-681)

class _Sampler(torch.autograd.Function):
    @staticmethod
    def forward(ctx, planes_tm, palette, x, dec, heads: int, sr: float, inv_alpha: float, beta: float):
        lib = _lib.load()
        B, P = x.shape[0], x.shape[1]
        dev = x.device
        x_c = x.contiguous()
        pal = None if palette is None else palette.contiguous()
        sigma = torch.empty((B, P), device=dev)
        rgb = torch.empty((B, P, 3), device=dev)
        y = torch.empty((B, P, 11), device=dev)
        f = _Sampler._field(planes_tm, pal, dec, heads, sr, inv_alpha, beta)
        _lib.check(lib.nfi_sampler_forward(ctypes.byref(f), _ptr(x_c), B, P, _ptr(sigma), _ptr(rgb), _ptr(y),
                                           _stream(dev)), 'nfi_sampler_forward')
        ctx.save_for_backward(planes_tm, pal, x_c, dec)
        ctx.cfg = (heads, sr, inv_alpha, beta)
        return sigma, rgb, y

    @staticmethod
    def _field(planes_tm, pal, dec, heads, sr, inv_alpha, beta):
        return _lib.NfiField(planes=_ptr(planes_tm), sb=planes_tm.stride(0), sq=planes_tm.stride(1),
                             st=planes_tm.stride(3), R=planes_tm.shape[2], _pad=0, dec=_ptr(dec), palette=_ptr(pal),
                             inv_alpha=float(inv_alpha), beta=float(beta), scene_range=float(sr), heads=int(heads))

    @staticmethod
    def backward(ctx, g_sigma, g_rgb, g_y):
        lib = _lib.load()
        planes_tm, pal, x, dec = ctx.saved_tensors
        heads, sr, inv_alpha, beta = ctx.cfg
        B, P = x.shape[0], x.shape[1]
        dev = x.device
        f = _Sampler._field(planes_tm, pal, dec, heads, sr, inv_alpha, beta)
        d_planes = None
        if ctx.needs_input_grad[0]:
            d_planes = torch.zeros_like(planes_tm)
            if d_planes.stride() != planes_tm.stride():
                raise RuntimeError('nfi: d planes strides differ from the planes view (non-dense planes view)')
        chunks = int(lib.nfi_sampler_chunks(B, P))
        d_pal_part = torch.empty((chunks, 30), device=dev) if pal is not None else None
        d_x = torch.empty_like(x) if ctx.needs_input_grad[2] else None
        gs = None if g_sigma is None else g_sigma.contiguous()
        gr = None if g_rgb is None else g_rgb.contiguous()
        gy = None if g_y is None else g_y.contiguous()
        st = _stream(dev)
        _lib.check(lib.nfi_sampler_backward(ctypes.byref(f), _ptr(x), B, P, _ptr(gs), _ptr(gr), _ptr(gy),
                                            _ptr(d_planes), _ptr(d_pal_part), _ptr(d_x), st), 'nfi_sampler_backward')
        d_pal = None
        if pal is not None:
            d_pal = torch.empty((B, 30), device=dev)
            ws = torch.empty((B * 64 * 30,), device=dev)
            _lib.check(lib.nfi_segment_sum(_ptr(d_pal_part), B, chunks // B, 30, _ptr(d_pal), _ptr(ws), st),
                       'nfi_segment_sum')
            d_pal = d_pal.view(B, 10, 3)
        return d_planes, d_pal, d_x, None, None, None, None, None


SAMPLER_OUTPUTS = ('sdf_distance', 'sigma', 'rgb', 'normals', 'semantics', 'coords')


def make_sampler(field, scene_range: Optional[float] = None):
    """The `sampler(x_in, request_sampler_outputs=['sigma', 'rgb'])` closure of Generator.forward
    (generator.py:587-681) over an nfi.TriplaneField (planes [B,3,32,R,R], palette, decoder,
    alpha / beta, attention_values 10 or 0, use_sdf): x_in [B, ..., 3] world points (image b's
    points on image b's planes) -> dict with 'sigma' [B, N], 'rgb' [B, N, 3], 'sdf_distance'
    [B, N, 1], 'semantics' [B, N, 10] (softmax of the logits), 'normals' [B, ..., 3] (normalised
    d distance / d x_in, computed through the HIP backward; needs grad mode, :599-622) and
    'coords' (x_in).  scene_range defaults to nfi.configure()'s."""
    from .render import MAX_ATTENTION, _check_frozen, attention_padded, get_config
    if field.viewdir_mapper is not None:
        raise NotImplementedError('the view-direction closure needs per-ray inputs: use render()')
    sr = float(scene_range if scene_range is not None else get_config().scene_range)
    heads = ((HEAD_RGB_SIGMOID if field.attention_values == 0 else 0)
             | (0 if field.use_sdf else HEAD_NERF_DENSITY))
    planes_tm = planes_texel_major(field.planes)
    w2, b2, pal_padded = attention_padded(field)     # 1..9 attention values: padded to the kernels' 10
    nattn = int(field.attention_values)
    dec = pack_decoder(field.w1, field.b1, w2, b2, key_tensors=(field.w1, field.b1, field.w2, field.b2))
    palette = pal_padded if nattn else None
    inv_alpha = 1.0 / float(field.alpha) if field.use_sdf else 1.0
    beta = float(field.beta) if field.use_sdf else 0.1

    def sampler(x_in: torch.Tensor, request_sampler_outputs: Sequence[str] = ('sigma', 'rgb')):
        for o in request_sampler_outputs:
            assert o in SAMPLER_OUTPUTS, o
        _require_device(x_in)
        # the packed decoder carries no gradient: a trainable decoder raises, as in render()
        _check_frozen(field)
        out = {}
        bs = x_in.shape[0]
        normals = 'normals' in request_sampler_outputs
        if normals:
            if not field.use_sdf or not torch.is_grad_enabled():
                raise AssertionError('normals need an SDF field and grad mode (generator.py:599-601)')
            x_in = x_in.requires_grad_()
        x = x_in.reshape(bs, -1, 3)
        sigma, rgb, y = _Sampler.apply(planes_tm, palette, x, dec, heads, sr, inv_alpha, beta)
        dist = y[..., :1]
        if normals:
            g, = torch.autograd.grad(dist[..., 0].sum(), x_in, create_graph=False)
            out['normals'] = torch.nn.functional.normalize(g, dim=-1)
            sigma, rgb, y, dist = sigma.detach(), rgb.detach(), y.detach(), dist.detach()
            x_in = x_in.detach()
        if 'sdf_distance' in request_sampler_outputs:
            out['sdf_distance'] = dist
        if 'sigma' in request_sampler_outputs:
            out['sigma'] = sigma
        if 'coords' in request_sampler_outputs:
            out['coords'] = x_in
        if 'semantics' in request_sampler_outputs:
            assert field.attention_values > 0
            out['semantics'] = torch.softmax(y[..., 1:1 + nattn], dim=-1)
        if 'rgb' in request_sampler_outputs:
            out['rgb'] = rgb
        return out

    return sampler


def sampler(generator, ws, extra_model_inputs: Optional[dict] = None):
    """Generator.forward(..., request_model_outputs=['sampler']) (generator.py:407-686): the
    producer modules run as in render() (nfi.render.field_from_generator), the closure on HIP."""
    from .render import field_from_generator
    f = field_from_generator(generator, ws, (), extra_model_inputs or {})
    return make_sampler(f, float(generator.scene_range) if hasattr(generator, 'scene_range') else None)
