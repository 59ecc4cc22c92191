"""Shared helpers for the GPU parity tests: run the HIP renderer and the CPU oracle on the
same inputs and compare."""

import torch

import nfi
from oracle import render_oracle as orc


def rel_l2(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.norm()
    return float((a - b).norm() / den) if den > 0 else float((a - b).norm())


def run_hip(inp, meta, dev, debug=None, with_grad=True):
    """inp: dict of CPU tensors (planes, palette, w1, b1, w2, b2, alpha, beta, cam, focal?,
    center?, bbox?, u_coarse, u_fine, g_rgb, g_mask)."""
    nfi.configure(scene_range=float(meta['scene_range']), white_background=bool(meta['white_bg']),
                  fine_sampling=bool(meta.get('fine', 1)))
    ncg = bool(meta.get('force_no_cam_grad', 0))
    planes = inp['planes'].to(dev).requires_grad_(with_grad)
    nattn = int(meta.get('attention_values', 10))
    use_sdf = bool(meta.get('use_sdf', 1))
    palette = inp['palette'].to(dev).requires_grad_(with_grad) if nattn else None
    cam = inp['cam'].to(dev).requires_grad_(with_grad and not ncg)
    focal = inp.get('focal')
    if focal is not None:
        focal = focal.to(dev).requires_grad_(with_grad and not ncg)
    center = inp.get('center')
    bbox = inp.get('bbox')
    mapper = None
    if meta.get('use_viewdir', 0):
        from nfi.viewdir import ViewDirectionMapper
        mapper = ViewDirectionMapper(nattn if nattn else 3)
        mapper.load_state_dict({k[3:]: v for k, v in inp.items() if k.startswith('vd_')})
        mapper = mapper.to(dev).requires_grad_(False)
    nfi.configure(use_viewdir=mapper is not None)
    f = nfi.TriplaneField(planes=planes, palette=palette, w1=inp['w1'].to(dev), b1=inp['b1'].to(dev),
                          w2=inp['w2'].to(dev), b2=inp['b2'].to(dev),
                          alpha=float(inp['alpha']) if use_sdf else 1.0,
                          beta=float(inp['beta']) if use_sdf else 0.1,
                          attention_values=nattn, use_sdf=use_sdf, viewdir_mapper=mapper)
    rnd = bool(meta['randomize'])
    uc = inp['u_coarse'].to(dev) if rnd else None
    uf = inp['u_fine'].to(dev) if rnd else None
    rgb, depth, mask, _, _, _ = nfi.render(
        f, int(meta['H']), int(meta['W']), cam, focal, None if center is None else center.to(dev),
        None if bbox is None else bbox.to(dev), None, int(meta['S']), randomize=rnd,
        force_no_cam_grad=ncg, u_coarse=uc, u_fine=uf, debug=debug,
        depth_mode='zbuffer' if meta.get('zbuffer') else 'ray')
    out = {'rgb': rgb.detach().cpu(), 'depth': depth.detach().cpu(), 'mask': mask.detach().cpu()}
    if with_grad:
        loss = (rgb * inp['g_rgb'].to(dev)).sum() + (mask * inp['g_mask'].to(dev)).sum()
        loss.backward()
        torch.cuda.synchronize()
        out['d_planes'] = planes.grad.cpu()
        if palette is not None:
            out['d_palette'] = palette.grad.cpu()
        if cam.requires_grad:
            out['d_cam'] = cam.grad.cpu()
            if focal is not None:
                out['d_focal'] = focal.grad.cpu()
    return out


def run_oracle64(inp, meta, with_grad=True, return_intermediates=False, z_fine=None):
    """The oracle evaluated in float64 — the 'exact' answer both fp32 paths are measured against."""
    inp64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in inp.items()}
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return run_oracle(inp64, meta, with_grad, return_intermediates, z_fine=z_fine)
    finally:
        torch.set_default_dtype(prev)


def run_oracle(inp, meta, with_grad=True, return_intermediates=False, z_fine=None):
    ncg = bool(meta.get('force_no_cam_grad', 0))
    nattn = int(meta.get('attention_values', 10))
    vd = {k[3:]: v for k, v in inp.items() if k.startswith('vd_')} or None
    field = orc.Field(planes=inp['planes'].clone().requires_grad_(with_grad),
                      w1=inp['w1'], b1=inp['b1'], w2=inp['w2'], b2=inp['b2'],
                      palette=inp['palette'].clone().requires_grad_(with_grad) if nattn else None,
                      alpha=inp.get('alpha'), beta=inp.get('beta'), scene_range=float(meta['scene_range']),
                      attention_values=nattn, use_sdf=bool(meta.get('use_sdf', 1)), viewdir=vd)
    cam = inp['cam'].clone().requires_grad_(with_grad and not ncg)
    focal = inp.get('focal')
    if focal is not None:
        focal = focal.clone().requires_grad_(with_grad and not ncg)
    rnd = bool(meta['randomize'])
    res = orc.render(field, int(meta['H']), int(meta['W']), cam, focal, inp.get('center'), inp.get('bbox'),
                     int(meta['S']), randomize=rnd, white_background=bool(meta['white_bg']),
                     fine_sampling=bool(meta.get('fine', 1)), force_no_cam_grad=ncg,
                     u_coarse=inp['u_coarse'] if rnd else None, u_fine=inp['u_fine'] if rnd else None,
                     return_intermediates=return_intermediates, z_fine=z_fine,
                     zbuffer=bool(meta.get('zbuffer', 0)))
    rgb, depth, mask = res[:3]
    out = {'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach()}
    if return_intermediates:
        out['inter'] = res[3]
    if with_grad:
        loss = (rgb * inp['g_rgb']).sum() + (mask * inp['g_mask']).sum()
        loss.backward()
        out['d_planes'] = field.planes.grad
        if field.palette is not None:
            out['d_palette'] = field.palette.grad
        if cam.requires_grad:
            out['d_cam'] = cam.grad
            if focal is not None:
                out['d_focal'] = focal.grad
    return out


def synthetic_inputs(B, H, W, S, R, scene_range, seed, ortho=False, flipped=True, white_bg=False,
                     randomize=True):
    """Seeded synthetic inversion inputs: planes N(0, 1.87^2), random-init decoder
    with the -0.97 SDF bias shift, palette wide_sigmoid_rescaled(N(0,1)), cameras on a sphere of
    radius 3.3*scene_range (focal 1.859)."""
    g = torch.Generator().manual_seed(seed)
    inp = {
        'planes': 1.87 * torch.randn(B, 3, 32, R, R, generator=g),
        'w1': torch.randn(64, 32, generator=g), 'b1': torch.zeros(64),
        'w2': torch.randn(11, 64, generator=g), 'b2': torch.zeros(11),
        'palette': orc.wide_sigmoid_rescaled(torch.randn(B, 10, 3, generator=g)),
        'alpha': torch.tensor([1.0]), 'beta': torch.tensor([0.1]),
    }
    inp['b2'][0] -= 0.97
    q = torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=-1)
    t2 = 0.05 * torch.randn(B, 2, generator=g)
    if ortho:
        s = torch.full((B, 1), 1.0 / scene_range)
        cam, focal = orc.pose_to_matrix(None, t2, s, q, flipped)
    else:
        f = 2 * 1.859
        s = torch.full((B,), f / (3.3 * scene_range))
        z0 = torch.full((B,), float(torch.log(torch.tensor(f - 1))))
        cam, focal = orc.pose_to_matrix(z0, t2, s, q, flipped)
        inp['focal'] = focal.detach()
    inp['cam'] = cam.detach()
    inp['u_coarse'] = torch.rand(B, H, W, S, generator=g)
    inp['u_fine'] = torch.rand(B * H * W, S, generator=g)
    inp['g_rgb'] = torch.randn(B, H, W, 3, generator=g)
    inp['g_mask'] = torch.randn(B, H, W, generator=g)
    meta = dict(H=H, W=W, S=S, R=R, scene_range=scene_range, white_bg=int(white_bg),
                randomize=int(randomize), force_no_cam_grad=0)
    return inp, meta


def run_hip_extras(inp, meta, dev):
    """nfi.render with compute_normals / compute_semantics / compute_coords (eval outputs)."""
    nfi.configure(scene_range=float(meta['scene_range']), white_background=bool(meta['white_bg']),
                  fine_sampling=True)
    mapper = None
    if any(k.startswith('vd_') for k in inp):
        from nfi.viewdir import ViewDirectionMapper
        mapper = ViewDirectionMapper(10)
        mapper.load_state_dict({k[3:]: v for k, v in inp.items() if k.startswith('vd_')})
        mapper = mapper.to(dev).requires_grad_(False)
    nfi.configure(use_viewdir=mapper is not None)
    f = nfi.TriplaneField(planes=inp['planes'].to(dev), palette=inp['palette'].to(dev),
                          w1=inp['w1'].to(dev), b1=inp['b1'].to(dev), w2=inp['w2'].to(dev),
                          b2=inp['b2'].to(dev), alpha=float(inp['alpha']), beta=float(inp['beta']),
                          viewdir_mapper=mapper)
    with torch.no_grad():
        rgb, depth, mask, nmap, smap, _ = nfi.render(
            f, int(meta['H']), int(meta['W']), inp['cam'].to(dev), inp['focal'].to(dev), None, None, None,
            int(meta['S']), randomize=True, compute_normals=bool(meta['compute_normals']),
            compute_semantics=bool(meta['compute_semantics']), compute_coords=bool(meta['compute_coords']),
            force_no_cam_grad=True, u_coarse=inp['u_coarse'].to(dev), u_fine=inp['u_fine'].to(dev))
    out = {'rgb': rgb.cpu(), 'depth': depth.cpu(), 'mask': mask.cpu()}
    if nmap is not None:
        out['normals'] = nmap.cpu()
    if smap is not None:
        out['semantics'] = smap.cpu()
    return out


def run_oracle_extras(inp, meta, dtype=torch.float32):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        cast = {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in inp.items()}
        field = orc.Field(planes=cast['planes'], w1=cast['w1'], b1=cast['b1'], w2=cast['w2'], b2=cast['b2'],
                          palette=cast['palette'], alpha=cast['alpha'], beta=cast['beta'],
                          scene_range=float(meta['scene_range']),
                          viewdir={k[3:]: v for k, v in cast.items() if k.startswith('vd_')} or None)
        rgb, depth, mask, nmap, smap = orc.render(
            field, int(meta['H']), int(meta['W']), cast['cam'], cast['focal'], None, None, int(meta['S']),
            randomize=True, white_background=bool(meta['white_bg']), force_no_cam_grad=True,
            u_coarse=cast['u_coarse'], u_fine=cast['u_fine'], compute_normals=bool(meta['compute_normals']),
            compute_semantics=bool(meta['compute_semantics']), compute_coords=bool(meta['compute_coords']))
    finally:
        torch.set_default_dtype(prev)
    out = {'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach()}
    if nmap is not None:
        out['normals'] = nmap.detach()
    if smap is not None:
        out['semantics'] = smap.detach()
    return out
