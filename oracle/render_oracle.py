"""CPU ORACLE for the nfi volume renderer — TEST INFRASTRUCTURE ONLY.

This module is a plain-PyTorch (fp32, CPU) restatement of the reference renderer of
yuliangguo/nerf-from-image (reference @ 2024-10-08).  It exists to CHECK the HIP product
path and to serve as bench.py's `cpu_baseline` leg.  It is never imported by the product
package (`nerf-from-image_amd/nfi`): only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s cpu_baseline leg may use it.

Pinning: every function below restates the reference function cited in its docstring
(op for op, same op order).  The restatement is pinned against golden vectors produced by
running the reference's own code in the build container (`tests/golden/gen_golden.py`
imports /root/reference and AST-extracts `render` from run.py:176-350); see
`tests/test_oracle_golden.py`.  The reference publishes no tests of its own.

Extension over the reference (for parity testing only): the random draws of the
stratified sampler (nerf_utils.py:118-120) and of sample_pdf (nerf_utils.py:202-205) can be
INJECTED (`u_coarse`, `u_fine`).  When they are not injected the draws happen in exactly the
reference's order (torch.rand_like, then torch.rand), so a seeded oracle equals a seeded
reference bit for bit.
"""

from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass
from typing import Optional


import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------------------
# lib/nerf_utils.py
# --------------------------------------------------------------------------------------

def cumprod_exclusive(tensor: torch.Tensor) -> torch.Tensor:
    """nerf_utils.py:20-25 (tf.math.cumprod(exclusive=True))."""
    cumprod = torch.cumprod(tensor[..., :-1], dim=-1)
    return torch.cat((torch.ones_like(cumprod[..., :1]), cumprod), dim=-1)


def get_ray_bundle(height: int, width: int, focal_length: Optional[torch.Tensor],
                   tform_cam2world: torch.Tensor, bbox: Optional[torch.Tensor],
                   center: Optional[torch.Tensor] = None):
    """nerf_utils.py:28-93.  Pixel grid arange(W)/W (corner, no +0.5); perspective branch
    (:40-66) with optional `center` (:43-47) and `bbox` (:52-56); ortho branch (:67-91)."""
    dev = tform_cam2world.device
    ii, jj = torch.meshgrid(torch.arange(width, device=dev) / width,
                            torch.arange(height, device=dev) / height, indexing='xy')
    if focal_length is not None:
        if center is not None:
            ii = ii.unsqueeze(0) - 0.5 * (2 * center[:, 0, None, None] - 1) - 0.5
            jj = jj.unsqueeze(0) - 0.5 * (2 * center[:, 1, None, None] - 1) - 0.5
        else:
            ii = ii.unsqueeze(0) - 0.5
            jj = jj.unsqueeze(0) - 0.5
        if bbox is not None:
            ii = (bbox[:, 1:2, 0].unsqueeze(-1) * (ii + 0.5) + bbox[:, 0:1, 0].unsqueeze(-1)) * 0.5
            jj = -(bbox[:, 1:2, 1].unsqueeze(-1) * (-jj + 0.5) + bbox[:, 0:1, 1].unsqueeze(-1)) * 0.5
        ii = ii / focal_length.unsqueeze(-1).unsqueeze(-1)
        jj = jj / focal_length.unsqueeze(-1).unsqueeze(-1)
        directions = torch.stack((ii, -jj, -torch.ones_like(ii)), dim=-1)
        ray_directions = torch.sum(directions[..., None, :] * tform_cam2world[:, None, None, :3, :3], dim=-1)
        ray_origins = tform_cam2world[:, None, None, :3, -1].expand(ray_directions.shape)
    else:
        ii = (ii.unsqueeze(0) - 0.5) * 2
        jj = (jj.unsqueeze(0) - 0.5) * 2
        if bbox is not None:
            ii = (bbox[:, 1:2, 0].unsqueeze(-1) * (ii / 2 + 0.5) + bbox[:, 0:1, 0].unsqueeze(-1))
            jj = -(bbox[:, 1:2, 1].unsqueeze(-1) * (-jj / 2 + 0.5) + bbox[:, 0:1, 1].unsqueeze(-1))
        origins = torch.stack((ii, -jj, torch.zeros_like(ii)), dim=-1)
        directions = torch.stack((torch.zeros_like(ii), torch.zeros_like(ii), -torch.ones_like(ii)), dim=-1)
        ray_origins = (torch.sum(origins[..., None, :] * tform_cam2world[:, None, None, :3, :3], dim=-1)
                       + tform_cam2world[:, None, None, :3, -1])
        ray_directions = (torch.sum(directions[..., None, :] * tform_cam2world[:, None, None, :3, :3], dim=-1)
                          / tform_cam2world[:, None, None, 3, 3].unsqueeze(-1))
    return ray_origins, ray_directions


def compute_query_points_from_rays(ray_origins, ray_directions, near_thresh, far_thresh,
                                   num_samples: int, randomize: bool = True,
                                   u: Optional[torch.Tensor] = None):
    """nerf_utils.py:96-122.  `u` (same shape as depth_values) replaces torch.rand_like."""
    near_plane = near_thresh.unsqueeze(-1)
    far_plane = far_thresh.unsqueeze(-1)
    depth_values = torch.lerp(near_plane, far_plane,
                              torch.arange(num_samples, device=ray_origins.device) / num_samples)
    if len(depth_values.shape) != 4:
        depth_values = depth_values[:, None, None, :]
        near_plane = near_plane[:, None, None, :]
        far_plane = far_plane[:, None, None, :]
    if randomize:
        delta = (far_plane - near_plane) / num_samples
        if u is None:
            u = torch.rand_like(depth_values)
        depth_values = depth_values + u * delta
    query_points = ray_origins[..., None, :] + ray_directions[..., None, :] * depth_values[..., :, None]
    return query_points, depth_values


def render_volume_density(sigma_a, rgb, ray_origins, ray_directions, depth_values,
                          white_background: bool = True, normals=None, semantics=None):
    """nerf_utils.py:125-163.  Returns (rgb, depth, mask) or, when normals / semantics are given,
    (rgb, depth, mask, normal_map, semantic_map) (normals composited with detached weights)."""
    zero_tensor = torch.zeros((1,), dtype=ray_origins.dtype, device=ray_origins.device)
    dists = torch.cat((depth_values[..., 1:] - depth_values[..., :-1],
                       zero_tensor.expand(depth_values[..., :1].shape)), dim=-1)
    dists = dists * ray_directions.norm(p=2, dim=-1, keepdim=True)
    alpha = 1. - torch.exp(-sigma_a * dists)
    weights = alpha * cumprod_exclusive(1. - alpha + 1e-10)
    rgb_map = (weights[..., None] * rgb).sum(dim=-2)
    depth_map = (weights.detach() * depth_values.detach()).sum(dim=-1)
    normal_map = (weights[..., None].detach() * normals).sum(dim=-2) if normals is not None else None
    semantic_map = (weights[..., None] * semantics).sum(dim=-2) if semantics is not None else None
    mask = weights.sum(-1)
    if white_background:
        rgb_map = rgb_map + (1. - mask[..., None])
        if normal_map is not None:
            normal_map = normal_map + (1. - mask[..., None])
    if normals is None and semantics is None:
        return rgb_map, depth_map, mask
    return rgb_map, depth_map, mask, normal_map, semantic_map


def render_volume_density_full(sigma_a, rgb, ray_origins, ray_directions, depth_values, normals=None,
                               semantics=None, white_background: bool = True):
    """nerf_utils.py:125-163 with the reference's own signature and 5-tuple return (the per-stage
    seam nfi.stages.render_volume_density is checked against it)."""
    out = render_volume_density(sigma_a, rgb, ray_origins, ray_directions, depth_values, white_background,
                                normals, semantics)
    if len(out) == 3:
        return out + (None, None)
    return out


def render_volume_density_weights_only(sigma_a, ray_origins, ray_directions, depth_values):
    """nerf_utils.py:166-182."""
    zero_tensor = torch.zeros((1,), dtype=ray_origins.dtype, device=ray_origins.device)
    dists = torch.cat((depth_values[..., 1:] - depth_values[..., :-1],
                       zero_tensor.expand(depth_values[..., :1].shape)), dim=-1)
    dists = dists * ray_directions.norm(p=2, dim=-1, keepdim=True)
    alpha = 1. - torch.exp(-sigma_a * dists)
    return alpha * cumprod_exclusive(1. - alpha + 1e-10)


def sample_pdf(bins, weights, num_samples: int, deterministic: bool = False,
               u: Optional[torch.Tensor] = None):
    """nerf_utils.py:185-224.  `u` ([rays, num_samples]) replaces torch.rand."""
    weights = weights + 1e-5
    pdf = weights / weights.sum(dim=-1, keepdim=True)
    cdf = torch.cumsum(pdf, dim=-1)
    cdf = torch.cat((torch.zeros_like(cdf[..., :1]), cdf), dim=-1)
    if deterministic:
        u = torch.linspace(0.0, 1.0, steps=num_samples, dtype=weights.dtype, device=weights.device)
        u = u.expand(list(cdf.shape[:-1]) + [num_samples])
    elif u is None:
        u = torch.rand(list(cdf.shape[:-1]) + [num_samples], dtype=weights.dtype, device=weights.device)
    u = u.contiguous()
    cdf = cdf.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.max(torch.zeros_like(inds - 1), inds - 1)
    above = torch.min((cdf.shape[-1] - 1) * torch.ones_like(inds), inds)
    inds_g = torch.stack((below, above), dim=-1)
    matched_shape = (inds_g.shape[0], inds_g.shape[1], cdf.shape[-1])
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(matched_shape), 2, inds_g)
    bins_g = torch.gather(bins.unsqueeze(1).expand(matched_shape), 2, inds_g)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    return bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])


def compute_near_far_planes(ray_origins, ray_directions, scene_range: float):
    """nerf_utils.py:227-275 (slab test; misses take the min near / max far over all hits)."""
    out_shape = ray_origins.shape[:-1]
    ray_origins = ray_origins.detach().reshape(-1, 3)
    ray_directions = ray_directions.detach().reshape(-1, 3)
    bvol = torch.tensor([[-scene_range] * 3, [scene_range] * 3], dtype=ray_origins.dtype,
                        device=ray_origins.device)
    invdir = 1 / ray_directions
    neg_sign = (invdir < 0).long()
    pos_sign = 1 - neg_sign
    xmin = (bvol[neg_sign[:, 0], 0] - ray_origins[:, 0]) * invdir[:, 0]
    xmax = (bvol[pos_sign[:, 0], 0] - ray_origins[:, 0]) * invdir[:, 0]
    ymin = (bvol[neg_sign[:, 1], 1] - ray_origins[:, 1]) * invdir[:, 1]
    ymax = (bvol[pos_sign[:, 1], 1] - ray_origins[:, 1]) * invdir[:, 1]
    zmin = (bvol[neg_sign[:, 2], 2] - ray_origins[:, 2]) * invdir[:, 2]
    zmax = (bvol[pos_sign[:, 2], 2] - ray_origins[:, 2]) * invdir[:, 2]
    mask = torch.ones(ray_origins.shape[:-1], dtype=torch.bool, device=ray_origins.device)
    mask[(xmin > ymax) | (ymin > xmax)] = False
    near_plane = torch.max(xmin, ymin)
    far_plane = torch.min(xmax, ymax)
    mask[(near_plane > zmax) | (zmin > far_plane)] = False
    near_plane = torch.max(near_plane, zmin)
    far_plane = torch.min(far_plane, zmax)
    near_plane[~mask] = near_plane[mask].min()
    far_plane[~mask] = far_plane[mask].max()
    near_plane.clamp_(min=0.1)
    far_plane.clamp_(min=0.1)
    eps = 1e-3
    mask_eps = (far_plane - near_plane) < eps
    far_plane[mask_eps] = near_plane[mask_eps] + eps
    return near_plane.reshape(out_shape), far_plane.reshape(out_shape)


# --------------------------------------------------------------------------------------
# models/generator.py + models/stylegan.py (the radiance field evaluated per point)
# --------------------------------------------------------------------------------------

def laplace_cdf(x, beta):
    """generator.py:30-33."""
    return 0.5 + 0.5 * torch.sign(x) * (1 - torch.exp(-x.abs() / beta))


def wide_sigmoid_rescaled(x):
    """generator.py:36-39."""
    return torch.sigmoid(x) * 2.004 - 1.002


def equalized_linear(x, weight, bias, lr_multiplier: float = 1.0):
    """stylegan.py:148-180 (EqualizedLinear.forward, activate=False)."""
    weight_gain = lr_multiplier / math.sqrt(weight.shape[1])
    return F.linear(x, weight * weight_gain, bias * lr_multiplier)


@dataclass
class Field:
    """Everything the renderer reads from the Generator (generator.py:392-399, 475-503):
    planes [b,3,32,R,R] (synthesis output viewed at generator.py:476-477), the
    TriplanarDecoder's two EqualizedLinear layers (raw parameters, generator.py:295-299),
    the per-image attention palette [b,10,3] (AttentionMapper output, generator.py:455-462),
    and the SDF parameters alpha, beta (generator.py:397-399).  attention_values = 0 (no
    palette; decoder [4, 64]: distance + 3 colour features, generator.py:377-384) and
    use_sdf = False (no alpha / beta) are the reference's other field variants."""
    planes: torch.Tensor
    w1: torch.Tensor       # [64, 32]
    b1: torch.Tensor       # [64]
    w2: torch.Tensor       # [11, 64] ([4, 64] without attention)
    b2: torch.Tensor       # [11]
    palette: Optional[torch.Tensor]  # [b, 10, 3] (None without attention)
    alpha: Optional[torch.Tensor]    # [1] (None without SDF)
    beta: Optional[torch.Tensor]     # [1]
    scene_range: float
    attention_values: int = 10
    use_sdf: bool = True
    viewdir: Optional[dict] = None   # --use_viewdir: ViewDirectionMapper parameters (state_dict keys)


def viewdir_trunk(params: dict, viewdir):
    """ViewDirectionMapper.forward generator.py:223-238 (the per-ray trunk): viewdir [..., 1, 3]
    -> x [..., 1, 32].  fc1..fc4 have no bias; LayerNorm eps 1e-5 with affine parameters."""
    def lin(x, name):
        return equalized_linear(x, params[f'{name}.weight'], params.get(f'{name}.bias',
                                                                         torch.zeros(params[f'{name}.weight'].shape[0],
                                                                                     dtype=x.dtype)))

    def norm(x, name):
        return F.layer_norm(x, (x.shape[-1],), params[f'{name}.weight'], params[f'{name}.bias'], 1e-5)

    scale = math.sqrt(2) / 2
    relu = lambda t: F.leaky_relu(t, 0.2)  # noqa: E731
    x = relu(lin(viewdir, 'fc0'))
    shortcut = x
    x = relu(norm(lin(x, 'fc1'), 'norm1'))
    x = relu(norm(lin(x, 'fc2'), 'norm2'))
    x = (x + shortcut) * scale
    shortcut = x
    x = relu(norm(lin(x, 'fc3'), 'norm3'))
    x = relu(norm(lin(x, 'fc4'), 'norm4'))
    x = (x + shortcut) * scale
    x = relu(lin(x, 'fc5'))
    return lin(x, 'fc6')


def viewdir_closure(params: dict, x, features):
    """mapper_closure generator.py:242-250: output(leaky_relu(x + features)) with x [b,H,W,1,32]
    broadcast over each ray's samples."""
    shape = features.shape
    f = features.view(*x.shape[:-2], -1, x.shape[-1])
    y = F.leaky_relu(x + f, 0.2).view(shape)
    return equalized_linear(y, params['output.weight'], params['output.bias'])


def triplanar_decoder(planes, coords, w1, b1, w2, b2):
    """TriplanarDecoder.forward generator.py:301-331, non-double-backward branch (:311-326)."""
    xy, xz, yz = planes[:, 0], planes[:, 1], planes[:, 2]
    nf = xy.shape[1]
    e1 = F.grid_sample(xy, coords[..., [0, 1]], mode='bilinear', padding_mode='border', align_corners=True)
    e2 = F.grid_sample(xz, coords[..., [0, 2]], mode='bilinear', padding_mode='border', align_corners=True)
    e3 = F.grid_sample(yz, coords[..., [1, 2]], mode='bilinear', padding_mode='border', align_corners=True)
    x = (e1 + e2 + e3) / 3
    x = x.view(x.shape[0], nf, -1).transpose(-2, -1)
    h = F.softplus(equalized_linear(x, w1, b1))           # net[0], net[1]  (generator.py:295-299)
    x = equalized_linear(h, w2, b2)                        # net[2]
    return x[..., 1:], x[..., :1]                          # features, density_or_distance


def sampler(field: Field, x_in, extras=(), xray=None):
    """The `sampler` closure generator.py:587-681 (with field.viewdir: the view-direction mapper
    closure on the features, :661-663, xray = its per-ray trunk output); use_sdf=True,
    attention_values=10 is the inversion configuration (the other density / colour heads follow
    field.use_sdf / field.attention_values).  Returns (sigma, rgb), or with `extras` ⊂
    {'normals','semantics','coords'} (sigma, rgb, dict): normals = normalize(d distance / d x_in)
    by autograd (create_graph=False; sigma and rgb are then detached, :599-622), semantics = the
    softmax probabilities (:672-674), coords = x_in (:643-644)."""
    out = {}
    if 'normals' in extras:
        x_in = x_in.detach().requires_grad_()
    bs = x_in.shape[0]
    x = x_in.view(bs, -1, 1, 3) / field.scene_range
    with torch.no_grad():
        mask = (x.abs() > 1).any(dim=-1).float()
        mask = mask.flatten(1, len(mask.shape) - 1)
    with torch.enable_grad() if 'normals' in extras else contextlib.nullcontext():
        features, density_or_distance = triplanar_decoder(field.planes, x, field.w1, field.b1, field.w2,
                                                          field.b2)
    if 'normals' in extras:
        x_grad, = torch.autograd.grad(density_or_distance[..., -1].sum(), x_in, create_graph=False)
        out['normals'] = F.normalize(x_grad, dim=-1)
        density_or_distance = density_or_distance.detach()
        features = features.detach()
        x_in = x_in.detach()
    if 'coords' in extras:
        out['coords'] = x_in
    if field.use_sdf:                                        # generator.py:628-636
        beta = field.beta
        alpha = 1 / field.alpha
        neg_distance = -density_or_distance[..., -1]
        density_prealpha = laplace_cdf(neg_distance, beta) * (1 - mask)
        sigma = alpha * density_prealpha
    else:                                                    # standard NeRF density, :637-641
        density_pre = density_or_distance[..., -1] - 1
        sigma = F.softplus(density_pre) * (1 - mask)
    if field.viewdir is not None:                            # :661-663
        features = viewdir_closure(field.viewdir, xray, features)
    if field.attention_values == 0:                          # :665-666
        rgb = wide_sigmoid_rescaled(features)
    else:
        attention_probs = F.softmax(features, dim=-1)
        if 'semantics' in extras:
            out['semantics'] = attention_probs
        rgb = torch.matmul(attention_probs, field.palette)
    if extras:
        return sigma, rgb, out
    return sigma, rgb


def sampler_with_distance(field: Field, x_in):
    """The sampler closure's 'sigma', 'rgb' and 'sdf_distance' outputs (generator.py:587-681):
    sigma [b,N], rgb [b,N,3], density_or_distance [b,N,1] (the per-stage seam
    nfi.stages.make_sampler is checked against it)."""
    bs = x_in.shape[0]
    x = x_in.view(bs, -1, 1, 3) / field.scene_range
    with torch.no_grad():
        mask = (x.abs() > 1).any(dim=-1).float()
        mask = mask.flatten(1, len(mask.shape) - 1)
    features, dist = triplanar_decoder(field.planes, x, field.w1, field.b1, field.w2, field.b2)
    if field.use_sdf:
        sigma = (1 / field.alpha) * (laplace_cdf(-dist[..., -1], field.beta) * (1 - mask))
    else:
        sigma = F.softplus(dist[..., -1] - 1) * (1 - mask)
    if field.attention_values == 0:
        rgb = wide_sigmoid_rescaled(features)
    else:
        rgb = torch.matmul(F.softmax(features, dim=-1), field.palette)
    return sigma, rgb, dist


# --------------------------------------------------------------------------------------
# run.py:176-350 — render()
# --------------------------------------------------------------------------------------

def render(field: Field, height: int, width: int, tform_cam2world, focal_length, center, bbox,
           depth_samples_per_ray: int, randomize: bool = True, white_background: bool = False,
           fine_sampling: bool = True, force_no_cam_grad: bool = False,
           u_coarse: Optional[torch.Tensor] = None, u_fine: Optional[torch.Tensor] = None,
           return_intermediates: bool = False, compute_normals: bool = False,
           compute_semantics: bool = False, compute_coords: bool = False,
           z_fine: Optional[torch.Tensor] = None, zbuffer: bool = False):
    """run.py:176-350 (args.use_viewdir = field.viewdir is not None).  Returns (rgb [b,H,W,3], depth [b,H,W],
    mask [b,H,W]) (+ intermediates dict); with any compute_* flag (run.py:227-257, 293-335)
    (rgb, depth, mask, normal_map [b,H,W,3] | None, semantic_map [b,H,W,10 | 3] | None) — the
    coords map replaces the semantic map when compute_coords (run.py:334-335)."""
    extras = tuple(n for n, f in (('normals', compute_normals), ('semantics', compute_semantics),
                                  ('coords', compute_coords)) if f)
    ray_origins, ray_directions = get_ray_bundle(height, width, focal_length, tform_cam2world, bbox, center)
    ray_directions = F.normalize(ray_directions, dim=-1)
    with torch.no_grad():
        near_thresh, far_thresh = compute_near_far_planes(ray_origins.detach(), ray_directions.detach(),
                                                          field.scene_range)
    query_points, depth_values = compute_query_points_from_rays(
        ray_origins, ray_directions, near_thresh, far_thresh, depth_samples_per_ray,
        randomize=randomize, u=u_coarse)
    if force_no_cam_grad:
        query_points = query_points.detach()
        depth_values = depth_values.detach()
        ray_directions = ray_directions.detach()
    xray = None
    if field.viewdir is not None:                            # run.py:216-219, generator.py:464-465
        xray = viewdir_trunk(field.viewdir, ray_directions.unsqueeze(-2))
    ex = {}
    if extras:
        sigma, rgb, ex = sampler(field, query_points, extras, xray=xray)
    else:
        sigma, rgb = sampler(field, query_points, xray=xray)
    sigma = sigma.view(*query_points.shape[:-1], -1)
    rgb = rgb.view(*query_points.shape[:-1], -1)
    ex = {k: v.view(*query_points.shape[:-1], -1) for k, v in ex.items()}
    inter = {'near': near_thresh, 'far': far_thresh, 'z_coarse': depth_values,
             'ro': ray_origins.detach(), 'rd': ray_directions.detach()}
    if fine_sampling:
        z_vals = depth_values
        with torch.no_grad():
            weights = render_volume_density_weights_only(sigma.squeeze(-1), ray_origins, ray_directions,
                                                         depth_values).flatten(0, 2)
            weights = F.max_pool1d(weights.unsqueeze(1).float(), 2, 1, padding=1)
            weights = F.avg_pool1d(weights, 2, 1).squeeze()
            weights = weights + 0.01
            z_vals_mid = .5 * (z_vals[..., 1:] + z_vals[..., :-1])
            z_samples = sample_pdf(z_vals_mid.flatten(0, 2), weights[..., 1:-1], depth_samples_per_ray,
                                   deterministic=not randomize, u=u_fine)
            if z_fine is not None:      # (tests: evaluate at given fine depths [b*H*W, S] instead)
                z_samples = z_fine.to(z_samples.dtype).reshape(z_samples.shape)
            z_samples = z_samples.view(*z_vals.shape[:3], z_samples.shape[-1])
        z_values_sorted, z_indices_sorted = torch.sort(torch.cat((z_vals, z_samples), dim=-1), dim=-1)
        query_points_fine = ray_origins[..., None, :] + ray_directions[..., None, :] * z_samples[..., :, None]
        ex_fine = {}
        if extras:
            sigma_fine, rgb_fine, ex_fine = sampler(field, query_points_fine, extras, xray=xray)
        else:
            sigma_fine, rgb_fine = sampler(field, query_points_fine, xray=xray)
        sigma_fine = sigma_fine.view(*query_points_fine.shape[:-1], -1)
        rgb_fine = rgb_fine.view(*query_points_fine.shape[:-1], -1)

        def merge(a, b):
            return torch.cat((a, b), dim=-2).gather(
                -2, z_indices_sorted.unsqueeze(-1).expand(-1, -1, -1, -1, a.shape[-1]))
        sigma = merge(sigma, sigma_fine)
        rgb = merge(rgb, rgb_fine)
        ex = {k: merge(v, ex_fine[k].view(*query_points_fine.shape[:-1], -1)) for k, v in ex.items()}
        depth_values = z_values_sorted
        inter['z_fine'] = z_samples
    inter['z_sorted'] = depth_values
    inter['sigma'] = sigma.squeeze(-1)
    inter['rgb'] = rgb
    if extras:
        semantics = ex.get('coords', ex.get('semantics'))
        outs = render_volume_density(sigma.squeeze(-1), rgb, ray_origins, ray_directions, depth_values,
                                     white_background=white_background, normals=ex.get('normals'),
                                     semantics=semantics)
        if outs[3] is None and outs[4] is None:
            outs = outs[:3]
        if len(outs) == 3:
            outs = (*outs, None, None)
        return (*outs, inter) if return_intermediates else outs
    rgb_map, depth_map, mask = render_volume_density(sigma.squeeze(-1), rgb, ray_origins, ray_directions,
                                                     depth_values, white_background=white_background)
    if zbuffer:
        depth_map = zbuffer_depth(depth_map, ray_directions, tform_cam2world)
    if return_intermediates:
        return rgb_map, depth_map, mask, inter
    return rgb_map, depth_map, mask


# --------------------------------------------------------------------------------------
# lib/pose_utils.py:48-75 — caller-side camera construction (used to build test cameras)
# --------------------------------------------------------------------------------------

def invert_space(mat):
    """pose_utils.py:20-27."""
    out_mat = torch.zeros_like(mat)
    out_mat[:, :3, :3] = mat[:, :3, :3].transpose(-2, -1) / mat[:, 3:4, 3:4]
    out_mat[:, 3, 3] = 1
    out_mat[:, :3, 3] = -torch.sum(mat[:, :3, :3] / mat[:, 3:4, 3:4] * mat[:, :3, None, 3], dim=-2)
    return out_mat


def zbuffer_depth(depth_predicted, ray_directions, tform_cam2world):
    """eval_nusc_persp.py:221-228 (the perspective eval scripts' render copy): ray distance ->
    camera-space z of the flipped camera."""
    tform_world2cam = invert_space(tform_cam2world)
    view_directions = torch.sum(ray_directions[..., None, :] * tform_world2cam[:, None, None, :3, :3], dim=-1)
    view_points3D = view_directions * depth_predicted.unsqueeze(-1)
    return view_points3D[..., -1] * (-1)


def quaternion_to_matrix(q):
    """pose_utils.py:30-45."""
    v = torch.eye(3, device=q.device).unsqueeze(0).expand(q.shape[0], -1, -1)
    qvec = q[:, 1:].unsqueeze(1).expand(-1, v.shape[1], -1)
    uv = torch.cross(qvec, v, dim=2)
    uuv = torch.cross(qvec, uv, dim=2)
    return v + 2 * (q[:, :1].unsqueeze(1) * uv + uuv)


def pose_to_matrix(z0, t2, s, q, camera_flipped: bool):
    """pose_utils.py:48-75."""
    R = quaternion_to_matrix(q)
    mat = torch.zeros((q.shape[0], 4, 4), device=R.device)
    mat[:, 3, 3] = 1
    mat[:, :3, :3] = R
    if z0 is not None:
        f = 1 + z0.exp()
        t3 = torch.cat((t2 / s.unsqueeze(-1), (f / s).unsqueeze(-1)), dim=-1)
        mat[:, :3, 3] = (t3[:, None, :] * R).sum(dim=-1)
        if camera_flipped:
            mat[:, :3, 1:] *= -1
        return mat, f / 2
    t3 = torch.cat((t2, torch.ones_like(t2[:, :1])), dim=-1) / s
    mat[:, :3, 3] = (t3[:, None, :] * R).sum(dim=-1)
    if camera_flipped:
        mat[:, :3, 1:] *= -1
    return mat, None
