"""Generate golden vectors by running the REFERENCE's own code (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
Needs /root/reference (read-only, imported, never copied).  Writes tests/golden/*.npz: inputs
and expected outputs/gradients of
  * render()  — AST-extracted verbatim from run.py:176-350 and executed with the reference's
                Generator (models/generator.py) whose synthesis network is replaced by a leaf
                tensor of small tri-planes (so the fixture stays small); the sampler closure,
                TriplanarDecoder (F.grid_sample), Laplace density, softmax colour head,
                nerf_utils ray bundle / near-far / stratified sampling / sample_pdf /
                compositing are all the reference's code;
  * per-stage nerf_utils functions (compute_near_far_planes, sample_pdf; seams.npz:
    cumprod_exclusive, get_ray_bundle, compute_query_points_from_rays,
    render_volume_density_weights_only in fp32 and fp64 with input gradients).
  * the producer: the reference Generator (mapping network, StyleGAN2
    synthesis network, AttentionMapper) at full size with seeded weights (golden_io.load_seeded,
    so no weights are stored), sampled planes + checksums, palette, and the latent gradient;
  * pose_utils pose_to_matrix / matrix_to_pose on a few cameras;
  * augment_impl (run.py:720-797) on images, the inversion loss's augmentation;
  * metrics.psnr / iou and pose_utils.rotation_matrix_distance (inversion report metrics);
  * an inversion trajectory: the loop of run.py:1960-2310 restated around
    the reference's Generator, render() and pose_utils, L1 loss, 3 Adam steps.
Random draws of the reference (torch.rand_like / torch.rand) are recovered by re-seeding and
drawing the same shapes in the same order, and stored as `u_coarse` / `u_fine`.
"""

import ast
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from lib import nerf_utils, pose_utils  # noqa: E402  (reference modules)
from models import generator  # noqa: E402

sys.path.insert(0, os.path.dirname(OUT))
from golden_io import load_seeded  # noqa: E402  (the seeded-weights recipe the tests share)


def extract_render(args_ns, dataset_config, path='run.py'):
    """`render` AST-extracted from run.py (or a script with its own copy, e.g. the perspective
    eval scripts' z-buffer variant eval_nusc_persp.py:43-231) and exec'd with its globals."""
    src = open(os.path.join(REF, path)).read()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'render'][0]
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {'torch': torch, 'F': F, 'nerf_utils': nerf_utils, 'pose_utils': pose_utils, 'args': args_ns,
          'dataset_config': dataset_config}
    exec(compile(mod, os.path.join(REF, path), 'exec'), ns)
    return ns['render']


class PlanesLeaf(torch.nn.Module):
    """Stand-in for stylegan.SynthesisNetwork: returns a leaf tensor of planes."""

    def __init__(self, planes):
        super().__init__()
        self.planes = planes

    def forward(self, ws, **kw):
        b = self.planes.shape[0]
        return self.planes.view(b, -1, self.planes.shape[-2], self.planes.shape[-1])


def make_cameras(b, scene_range, flipped, seed, ortho=False):
    g = torch.Generator().manual_seed(seed)
    q = F.normalize(torch.randn(b, 4, generator=g), dim=-1)
    focal = 1.859
    f = 2 * focal
    t2 = 0.05 * torch.randn(b, 2, generator=g)
    if ortho:
        s = torch.full((b,), 1.0 / scene_range) * (0.8 + 0.2 * torch.rand(b, generator=g))
        mat, fl = pose_utils.pose_to_matrix(None, t2, s, q, flipped)
        return mat, None
    s = torch.full((b,), f / (3.3 * scene_range))
    z0 = torch.full((b,), float(np.log(f - 1)))
    mat, fl = pose_utils.pose_to_matrix(z0, t2, s, q, flipped)
    return mat, fl


def render_case(name, seed, b, H, W, S, R, scene_range, white_bg, flipped, randomize,
                force_no_cam_grad=False, ortho=False, with_bbox=False, with_center=False,
                attention_values=10, use_sdf=True, render_file='run.py', use_viewdir=False,
                inside=False):
    torch.manual_seed(1000 + seed)
    gen = generator.Generator(512, scene_range, attention_values=attention_values, use_sdf=use_sdf,
                              use_viewdir=use_viewdir, disable_stylegan_noise=True)
    gen.eval()
    with torch.no_grad():
        if use_sdf:
            gen.decoder.net[2].bias[0] -= 0.97     # mask mean ~0.6 instead of ~5e-4
            gen.beta.fill_(0.1)
            gen.alpha.fill_(1.0)
        if use_viewdir:
            # the mapper's output layer is zero-initialised (generator.py:219-220) and its
            # LayerNorms are identity at init: seeded values so every term is exercised
            gv = torch.Generator().manual_seed(3000 + seed)
            for k, p in gen.viewdir_mapper.named_parameters():
                r = torch.randn(p.shape, generator=gv)
                p.copy_(1 + 0.2 * r if k.startswith('norm') and k.endswith('weight')
                        else 0.2 * r if k.endswith('bias') else r)
    planes = (1.87 * torch.randn(b, 3, 32, R, R)).requires_grad_()
    gen.synthesis_network = PlanesLeaf(planes)
    palette = generator.wide_sigmoid_rescaled(torch.randn(b, attention_values or 10, 3)).detach().requires_grad_()
    cam, focal = make_cameras(b, scene_range, flipped, seed, ortho=ortho)
    if inside:
        # nerf_utils.py:264-270: image 0's camera sits INSIDE the scene box (0.6 scene_range from
        # the centre, looking at it: near < 0 -> clamped to 0.1); image 1's camera is turned away
        # from the box (rotated 180 degrees about its y axis: the box lies behind it on every ray's
        # line, near and far < 0 -> both 0.1 -> far = near + 1e-3)
        cam = cam.detach().clone()
        t = cam[0, :3, 3]
        cam[0, :3, 3] = t * (0.6 * scene_range / float(t.norm()))
        cam[1, :3, 0] = -cam[1, :3, 0]
        cam[1, :3, 2] = -cam[1, :3, 2]
    cam = cam.detach().requires_grad_(not force_no_cam_grad)
    if focal is not None:
        focal = focal.detach().requires_grad_(not force_no_cam_grad)
    bbox = None
    center = None
    if with_bbox:
        bb = torch.tensor([[-0.1, -0.05], [1.9, 2.1]]).expand(b, 2, 2).clone()
        bbox = bb + 0.02 * torch.randn(b, 2, 2)
    if with_center:
        center = 0.5 + 0.05 * torch.randn(b, 2)
    ws = torch.zeros(b, 15, 512)
    args_ns = types.SimpleNamespace(use_viewdir=use_viewdir, fine_sampling=True, use_sdf=use_sdf,
                                    attention_values=attention_values)
    dataset_config = {'scene_range': scene_range, 'white_background': white_bg}
    render = extract_render(args_ns, dataset_config, render_file)

    rseed = 77 + seed
    torch.manual_seed(rseed)
    rgb, depth, mask, _, _, _ = render(gen, H, W, cam, focal, center, bbox, ws, S,
                                       randomize=randomize,
                                       extra_model_inputs=({'attention_values': palette}
                                                           if attention_values else {}),
                                       force_no_cam_grad=force_no_cam_grad)
    torch.manual_seed(rseed)
    if randomize:
        u_coarse = torch.rand(b, H, W, S)
        u_fine = torch.rand(b * H * W, S)
    else:
        u_coarse = torch.zeros(b, H, W, S)
        u_fine = torch.zeros(b * H * W, S)
    gseed = torch.Generator().manual_seed(5000 + seed)
    g_rgb = torch.randn(b, H, W, 3, generator=gseed)
    g_mask = torch.randn(b, H, W, generator=gseed)
    loss = (rgb * g_rgb).sum() + (mask * g_mask).sum()
    loss.backward()
    out = {
        'planes': planes.detach(), 'w1': gen.decoder.net[0].weight.detach(),
        'b1': gen.decoder.net[0].bias.detach(), 'w2': gen.decoder.net[2].weight.detach(),
        'b2': gen.decoder.net[2].bias.detach(),
        'cam': cam.detach(), 'u_coarse': u_coarse, 'u_fine': u_fine,
        'g_rgb': g_rgb, 'g_mask': g_mask,
        'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach(),
        'd_planes': planes.grad,
    }
    if attention_values:
        out['palette'], out['d_palette'] = palette.detach(), palette.grad
    if use_viewdir:
        out.update({f'vd_{k}': v.detach() for k, v in gen.viewdir_mapper.state_dict().items()})
    if use_sdf:
        out['alpha'], out['beta'] = gen.alpha.detach(), gen.beta.detach()
    if focal is not None:
        out['focal'] = focal.detach()
    if bbox is not None:
        out['bbox'] = bbox
    if center is not None:
        out['center'] = center
    if not force_no_cam_grad:
        out['d_cam'] = cam.grad
        if focal is not None:
            out['d_focal'] = focal.grad
    meta = dict(H=H, W=W, S=S, R=R, scene_range=scene_range, white_bg=int(white_bg),
                randomize=int(randomize), force_no_cam_grad=int(force_no_cam_grad),
                ortho=int(ortho), attention_values=attention_values, use_sdf=int(use_sdf),
                zbuffer=int(render_file != 'run.py'), use_viewdir=int(use_viewdir))
    np.savez_compressed(os.path.join(OUT, f'render_{name}.npz'),
                        **{k: v.numpy() for k, v in out.items()},
                        **{f'meta_{k}': np.array(v) for k, v in meta.items()})
    print(name, 'mask mean', float(mask.mean()), 'rgb mean', float(rgb.mean()))


def extras_case(name, seed, b, H, W, S, R, scene_range, white_bg, flipped, compute_normals,
                compute_semantics, compute_coords):
    """render() eval outputs (run.py:227-257, 293-335; generator.py:599-622, 643-644, 672-674;
    nerf_utils.py:146-161): normals (autograd d SDF / d point, normalised), semantics (softmax
    probabilities) and coords maps, composited like rgb.  No backward (eval-only outputs)."""
    torch.manual_seed(2000 + seed)
    gen = generator.Generator(512, scene_range, attention_values=10, use_sdf=True,
                              disable_stylegan_noise=True)
    gen.eval()
    with torch.no_grad():
        gen.decoder.net[2].bias[0] -= 0.97
        gen.beta.fill_(0.1)
        gen.alpha.fill_(1.0)
    planes = 1.87 * torch.randn(b, 3, 32, R, R)
    gen.synthesis_network = PlanesLeaf(planes)
    palette = generator.wide_sigmoid_rescaled(torch.randn(b, 10, 3)).detach()
    cam, focal = make_cameras(b, scene_range, flipped, 100 + seed)
    ws = torch.zeros(b, 15, 512)
    args_ns = types.SimpleNamespace(use_viewdir=False, fine_sampling=True, use_sdf=True,
                                    attention_values=10)
    dataset_config = {'scene_range': scene_range, 'white_background': white_bg}
    render = extract_render(args_ns, dataset_config)
    rseed = 177 + seed
    torch.manual_seed(rseed)
    rgb, depth, mask, normals, semantics, _ = render(
        gen, H, W, cam, focal, None, None, ws, S, randomize=True,
        extra_model_inputs={'attention_values': palette}, force_no_cam_grad=True,
        compute_normals=compute_normals, compute_semantics=compute_semantics,
        compute_coords=compute_coords)
    torch.manual_seed(rseed)
    u_coarse = torch.rand(b, H, W, S)
    u_fine = torch.rand(b * H * W, S)
    out = {
        'planes': planes, 'w1': gen.decoder.net[0].weight.detach(),
        'b1': gen.decoder.net[0].bias.detach(), 'w2': gen.decoder.net[2].weight.detach(),
        'b2': gen.decoder.net[2].bias.detach(), 'palette': palette,
        'alpha': gen.alpha.detach(), 'beta': gen.beta.detach(),
        'cam': cam.detach(), 'focal': focal.detach(), 'u_coarse': u_coarse, 'u_fine': u_fine,
        'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach(),
    }
    if normals is not None:
        out['normals'] = normals.detach()
    if semantics is not None:
        out['semantics'] = semantics.detach()
    meta = dict(H=H, W=W, S=S, R=R, scene_range=scene_range, white_bg=int(white_bg), randomize=1,
                force_no_cam_grad=1, ortho=0, compute_normals=int(compute_normals),
                compute_semantics=int(compute_semantics), compute_coords=int(compute_coords))
    np.savez_compressed(os.path.join(OUT, f'render_{name}.npz'),
                        **{k: v.numpy() for k, v in out.items()},
                        **{f'meta_{k}': np.array(v) for k, v in meta.items()})
    print(name, 'mask mean', float(mask.mean()))


def stage_cases():
    g = torch.Generator().manual_seed(123)
    # near/far: rays from a sphere around the box, some missing it (nerf_utils.py:227-275)
    n = 512
    ro = F.normalize(torch.randn(n, 3, generator=g), dim=-1) * 4.0
    tgt = torch.randn(n, 3, generator=g) * 1.2
    rd = F.normalize(tgt - ro, dim=-1)
    ro[:8] = torch.randn(8, 3, generator=g) * 0.3       # cameras inside the box (near clamped)
    near, far = nerf_utils.compute_near_far_planes(ro.view(8, 8, 8, 3), rd.view(8, 8, 8, 3), 1.4)
    # sample_pdf deterministic + random (nerf_utils.py:185-224)
    rays, S = 256, 32
    z = torch.sort(torch.rand(rays, S, generator=g) * 3 + 1, dim=-1)[0]
    bins = .5 * (z[:, 1:] + z[:, :-1])
    w = torch.rand(rays, S - 2, generator=g) ** 4
    w[:16] = 0.0                                          # degenerate (all-equal) pdfs
    det = nerf_utils.sample_pdf(bins, w, S, deterministic=True)
    torch.manual_seed(9)
    rnd = nerf_utils.sample_pdf(bins, w, S, deterministic=False)
    torch.manual_seed(9)
    u = torch.rand(rays, S)
    np.savez_compressed(os.path.join(OUT, 'stages.npz'),
                        nf_ro=ro.numpy(), nf_rd=rd.numpy(), nf_near=near.reshape(-1).numpy(),
                        nf_far=far.reshape(-1).numpy(),
                        pdf_bins=bins.numpy(), pdf_w=w.numpy(), pdf_det=det.numpy(),
                        pdf_u=u.numpy(), pdf_rnd=rnd.numpy())
    print('stages written')


def seam_cases():
    """The remaining nerf_utils seams as functions of their own (cumprod_exclusive :20-25,
    get_ray_bundle :28-93, compute_query_points_from_rays :96-122,
    render_volume_density_weights_only :166-182): outputs and input gradients in fp32 AND fp64 (the
    reference functions evaluated on double tensors), so the GPU tests can apply the 4x rule."""
    g = torch.Generator().manual_seed(321)
    out = {}

    def both(fn, inputs, grads):
        """outputs + VJPs of fn at fp32 and fp64 inputs (requires_grad where grads says)."""
        res = {}
        for dt, tag in ((torch.float32, '32'), (torch.float64, '64')):
            xs = [x.to(dt).clone().requires_grad_(rg) if x is not None else None for x, rg in inputs]
            ys = fn(*xs)
            ys = ys if isinstance(ys, tuple) else (ys,)
            loss = sum((y * gg.to(dt)).sum() for y, gg in zip(ys, grads) if gg is not None)
            loss.backward()
            res[tag] = ([y.detach().numpy() for y in ys],
                        [x.grad.numpy() if (x is not None and x.requires_grad) else None for x in xs])
        return res

    # cumprod_exclusive on rows with exact zeros / ones and long rows (several 64-lanes chunks)
    x = torch.rand(48, 150, generator=g) * 0.5 + 0.5
    x[:4, 10] = 0.0
    x[4:8, 70:] = 1.0
    x[8:12, -1] = 0.0                                      # the unused last input
    gx = torch.randn(48, 150, generator=g)
    r = both(nerf_utils.cumprod_exclusive, [(x, True)], [gx])
    out.update(cp_x=x.numpy(), cp_g=gx.numpy(), cp_out32=r['32'][0][0], cp_out64=r['64'][0][0],
               cp_dx32=r['32'][1][0], cp_dx64=r['64'][1][0])
    # get_ray_bundle: perspective, perspective + center + bbox, ortho + bbox
    B, H, W = 2, 6, 8
    for tag, persp, ctr, bb in (('p', True, False, False), ('pcb', True, True, True), ('ob', False, False, True)):
        cam = torch.eye(4).repeat(B, 1, 1)
        cam[:, :3, :3] = torch.linalg.qr(torch.randn(B, 3, 3, generator=g))[0]
        cam[:, :3, 3] = torch.randn(B, 3, generator=g) * 3
        if not persp:
            cam[:, 3, 3] = 0.5 + torch.rand(B, generator=g)
        focal = (1.5 + torch.rand(B, generator=g)) if persp else None
        center = torch.rand(B, 2, generator=g) if ctr else None
        bbox = (torch.rand(B, 2, 2, generator=g) - 0.5) if bb else None
        gro, grd = torch.randn(B, H, W, 3, generator=g), torch.randn(B, H, W, 3, generator=g)

        def fn(c, f, ce, bx):
            return nerf_utils.get_ray_bundle(H, W, f, c, bx, ce)
        r = both(fn, [(cam, True), (focal, persp), (center, False), (bbox, False)], [gro, grd])
        out.update({f'rb{tag}_cam': cam.numpy(), f'rb{tag}_gro': gro.numpy(), f'rb{tag}_grd': grd.numpy(),
                    f'rb{tag}_ro32': r['32'][0][0], f'rb{tag}_rd32': r['32'][0][1],
                    f'rb{tag}_ro64': r['64'][0][0], f'rb{tag}_rd64': r['64'][0][1],
                    f'rb{tag}_dcam32': r['32'][1][0], f'rb{tag}_dcam64': r['64'][1][0]})
        if persp:
            out.update({f'rb{tag}_focal': focal.numpy(), f'rb{tag}_dfocal32': r['32'][1][1],
                        f'rb{tag}_dfocal64': r['64'][1][1]})
        if ctr:
            out[f'rb{tag}_center'] = center.numpy()
        if bb:
            out[f'rb{tag}_bbox'] = bbox.numpy()
    # compute_query_points_from_rays: deterministic, and randomized with the draws recovered
    ro = torch.randn(2, 4, 5, 3, generator=g)
    rd = F.normalize(torch.randn(2, 4, 5, 3, generator=g), dim=-1)
    near = 0.5 + torch.rand(2, 4, 5, generator=g)
    far = near + 0.2 + 2 * torch.rand(2, 4, 5, generator=g)
    S = 20
    gp = torch.randn(2, 4, 5, S, 3, generator=g)
    for tag, rnd in (('d', False), ('r', True)):
        res = {}
        o, d = ro.clone().requires_grad_(), rd.clone().requires_grad_()
        torch.manual_seed(77)
        pts, depth = nerf_utils.compute_query_points_from_rays(o, d, near, far, S, randomize=rnd)
        (pts * gp).sum().backward()
        res['32'] = (pts.detach().numpy(), depth.detach().numpy(), o.grad.numpy(), d.grad.numpy())
        # fp64 truth (the reference's lerp rejects double inputs with its float arange weight): the same
        # depths in double, points and gradients of p = ro + rd t evaluated in fp64
        o64, d64 = ro.double().requires_grad_(), rd.double().requires_grad_()
        t64 = depth.detach().double()
        p64 = o64[..., None, :] + d64[..., None, :] * t64[..., :, None]
        (p64 * gp.double()).sum().backward()
        res['64'] = (p64.detach().numpy(), t64.numpy(), o64.grad.numpy(), d64.grad.numpy())
        torch.manual_seed(77)
        u = torch.rand(2, 4, 5, S)                       # rand_like(depth_values): the same draws
        out.update({f'qp{tag}_pts32': res['32'][0], f'qp{tag}_depth32': res['32'][1],
                    f'qp{tag}_dro32': res['32'][2], f'qp{tag}_drd32': res['32'][3],
                    f'qp{tag}_pts64': res['64'][0], f'qp{tag}_depth64': res['64'][1],
                    f'qp{tag}_dro64': res['64'][2], f'qp{tag}_drd64': res['64'][3], f'qp{tag}_u': u.numpy()})
    out.update(qp_ro=ro.numpy(), qp_rd=rd.numpy(), qp_near=near.numpy(), qp_far=far.numpy(), qp_g=gp.numpy())
    # render_volume_density_weights_only: densities with empty and opaque stretches
    N = 90
    t = torch.sort(torch.rand(2, 4, 5, N, generator=g) * 3 + 1, dim=-1)[0]
    sig = torch.relu(torch.randn(2, 4, 5, N, generator=g) * 3)
    sig[0, 0, :2] = 0.0                                  # empty rays
    sig[1, 1, :, 40:] = 50.0                             # opaque tails
    rdw = torch.randn(2, 4, 5, 3, generator=g)
    gw = torch.randn(2, 4, 5, N, generator=g)

    def wfn(sg, d, tt):
        return nerf_utils.render_volume_density_weights_only(sg, torch.zeros_like(d), d, tt)
    r = both(wfn, [(sig, True), (rdw, True), (t, True)], [gw])
    out.update(vw_sigma=sig.numpy(), vw_rd=rdw.numpy(), vw_t=t.numpy(), vw_g=gw.numpy(),
               vw_w32=r['32'][0][0], vw_w64=r['64'][0][0],
               vw_dsigma32=r['32'][1][0], vw_drd32=r['32'][1][1], vw_dt32=r['32'][1][2],
               vw_dsigma64=r['64'][1][0], vw_drd64=r['64'][1][1], vw_dt64=r['64'][1][2])
    np.savez_compressed(os.path.join(OUT, 'seams.npz'), **{k: v for k, v in out.items() if v is not None})
    print('seams written')


def extract_function(name, ns):
    """AST-extract a top-level function of run.py and exec it with the given globals."""
    src = open(os.path.join(REF, 'run.py')).read()
    fn = [n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name == name][0]
    exec(compile(ast.Module(body=[fn], type_ignores=[]), os.path.join(REF, 'run.py'), 'exec'), ns)
    return ns[name]


def metrics_cases():
    """metrics.psnr / iou (metrics.py:22-103, AST-extracted: the module imports lpips and
    scikit-image, absent here) and pose_utils.rotation_matrix_distance."""
    src = open(os.path.join(REF, 'lib', 'metrics.py')).read()
    ns = {'torch': torch}
    fns = [n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef)
           and n.name in ('range_check', 'psnr', 'iou')]
    exec(compile(ast.Module(body=fns, type_ignores=[]), os.path.join(REF, 'lib', 'metrics.py'), 'exec'), ns)
    g = torch.Generator().manual_seed(71)
    pred = torch.rand(4, 3, 16, 16, generator=g)
    tgt = (pred + 0.1 * torch.randn(4, 3, 16, 16, generator=g)).clamp(0, 1)
    tgt[3] = pred[3]                                        # the 60 dB clamp
    a0 = torch.rand(4, 16, 16, generator=g)
    a1 = torch.rand(4, 16, 16, generator=g)
    q = F.normalize(torch.randn(6, 4, generator=g), dim=-1)
    m0, _ = pose_utils.pose_to_matrix(None, torch.zeros(6, 2), torch.ones(1), q, False)
    q2 = F.normalize(q + 0.2 * torch.randn(6, 4, generator=g), dim=-1)
    m1, _ = pose_utils.pose_to_matrix(None, torch.zeros(6, 2), torch.ones(1), q2, False)
    np.savez_compressed(os.path.join(OUT, 'metrics.npz'), pred=pred.numpy(), tgt=tgt.numpy(),
                        psnr=ns['psnr'](pred, tgt, reduction='none').numpy(),
                        psnr_mean=ns['psnr'](pred, tgt).numpy(), a0=a0.numpy(), a1=a1.numpy(),
                        iou=ns['iou'](a0, a1, reduction='none').numpy(), m0=m0.numpy(),
                        m1=m1.numpy(), rot=pose_utils.rotation_matrix_distance(m0, m1).numpy())
    print('metrics written')


def augment_cases():
    """augment_impl (run.py:720-797) on images only, p=1 (the inversion loss's call)."""
    out = {}
    for wbg in (False, True):
        ns = {'torch': torch, 'F': F, 'np': np, 'pose_utils': pose_utils,
              'dataset_config': {'white_background': wbg},
              'args': types.SimpleNamespace(supervise_alpha=False)}
        augment_impl = extract_function('augment_impl', ns)
        g = torch.Generator().manual_seed(51 + wbg)
        img = torch.tanh(torch.randn(7, 6, 16, 12, generator=g))
        torch.manual_seed(61 + wbg)
        res, _, _, tform = augment_impl(img, None, None, 1.0)
        key = 'w' if wbg else 'b'
        out[f'{key}_img'] = img
        out[f'{key}_out'] = res
        out[f'{key}_rot'], out[f'{key}_scale'], out[f'{key}_translation'] = tform
    np.savez_compressed(os.path.join(OUT, 'augment.npz'), **{k: v.numpy() for k, v in out.items()},
                        meta_seed_b=np.array(61), meta_seed_w=np.array(62))
    print('augment written')


def seeded_generator(seed, scene_range=1.4):
    gen = generator.Generator(512, scene_range, attention_values=10, use_sdf=True,
                              disable_stylegan_noise=True)
    gen.eval()
    load_seeded(gen, seed)
    gen.requires_grad_(False)
    return gen


def producer_case(seed=21, b=2, nsample=8192):
    gen = seeded_generator(seed)
    sd = gen.state_dict()
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(b, 512, generator=g)
    ws = (0.6 * torch.randn(b, 15, 512, generator=g)).requires_grad_()
    with torch.no_grad():
        w_map = gen.mapping_network(z)
    palette = gen.texture_mapper(ws[:, 14])                       # generator.py:455-462
    planes = gen.synthesis_network(ws[:, :14])                    # generator.py:475-477
    gp = torch.randn(planes.shape, generator=torch.Generator().manual_seed(seed + 1))
    gq = torch.randn(palette.shape, generator=torch.Generator().manual_seed(seed + 2))
    ((planes * gp).sum() + (palette * gq).sum()).backward()
    idx = torch.randint(0, planes.numel(), (nsample,), generator=g)
    keys = list(sd.keys())
    shapes = json.dumps({k: list(v.shape) for k, v in sd.items()})
    np.savez_compressed(os.path.join(OUT, 'producer.npz'),
                        z=z.numpy(), ws=ws.detach().numpy(), w_map=w_map.numpy(),
                        palette=palette.detach().numpy(), idx=idx.numpy(),
                        planes_sample=planes.detach().reshape(-1)[idx].numpy(),
                        planes_chsum=planes.detach().double().sum(dim=(2, 3)).numpy(),
                        planes_chabs=planes.detach().double().abs().sum(dim=(2, 3)).numpy(),
                        d_ws=ws.grad.numpy(), sd_keys=np.array(keys), sd_shapes=np.array(shapes),
                        meta_seed=np.array(seed))
    print('producer planes std', float(planes.std()), 'palette mean', float(palette.mean()))


def ref_matrix_to_pose(mat, focal, flipped):
    """pose_utils.matrix_to_pose on float64 copies of the inputs: its matrix_to_quaternion
    (pose_utils.py:79, np.array(..., copy=False)) raises under numpy 2 unless handed float64;
    the outputs are cast back to float32 as the reference's float32 path returns them."""
    r = pose_utils.matrix_to_pose(mat.double(), None if focal is None else focal.double(), flipped)
    return tuple(None if v is None else v.float() for v in r)


def pose_cases():
    g = torch.Generator().manual_seed(31)
    out = {}
    for name, flipped, persp in (('pf', True, True), ('pu', False, True), ('of', True, False)):
        b = 4 if persp else 1      # pose_utils.py:69 divides [b,3] by s [b]: b=1 only
        q = F.normalize(torch.randn(b, 4, generator=g), dim=-1)
        t2 = 0.1 * torch.randn(b, 2, generator=g)
        s = 0.5 + torch.rand(b, generator=g)
        z0 = torch.randn(b, generator=g) if persp else None
        mat, focal = pose_utils.pose_to_matrix(z0, t2, s, q, flipped)
        rz0, rt2, rs, rq = ref_matrix_to_pose(mat, focal, flipped)
        out.update({f'{name}_q': q, f'{name}_t2': t2, f'{name}_s': s, f'{name}_mat': mat,
                    f'{name}_rt2': rt2, f'{name}_rs': rs, f'{name}_rq': rq})
        if persp:
            out.update({f'{name}_z0': z0, f'{name}_focal': focal, f'{name}_rz0': rz0})
    np.savez_compressed(os.path.join(OUT, 'pose.npz'), **{k: v.numpy() for k, v in out.items()})
    print('pose written')


def inversion_case(seed=41, b=2, H=16, S=8, steps=3, scene_range=1.4, flipped=True):
    """run.py:1960-2310 with --inv_loss l1, fine sampling, pose optimised; the loop skeleton
    is restated here, every op inside it is the reference's (Generator, render, pose_utils)."""
    gen = seeded_generator(seed, scene_range)
    with torch.no_grad():
        gen.decoder.net[2].bias[0] += SDF_SHIFT         # a partly-covered image (mask ~0.3-0.7)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        w_init = gen.mapping_network(torch.randn(64, 512, generator=g)).mean(dim=0, keepdim=True)
    cam0, focal0 = make_cameras(b, scene_range, flipped, seed)
    target = torch.tanh(torch.randn(b, H, H, 3, generator=g))
    args_ns = types.SimpleNamespace(use_viewdir=False, fine_sampling=True, use_sdf=True,
                                    attention_values=10)
    render = extract_render(args_ns, {'scene_range': scene_range, 'white_background': False})
    gain = 5.0
    z_ = (w_init.clone().expand(b, -1, -1).contiguous() / gain).requires_grad_()
    z0_, t2_, s_, R_ = ref_matrix_to_pose(cam0.detach(), focal0.detach(), flipped)
    for p in (t2_, s_, R_, z0_):
        p.requires_grad_()
    opt = torch.optim.Adam([z_, z0_, R_, s_, t2_], lr=2e-3, betas=(0.9, 0.95))
    u_c, u_f, losses, masks = [], [], [], []
    for it in range(steps):
        cam, focal = pose_utils.pose_to_matrix(z0_, t2_, s_, F.normalize(R_, dim=-1), flipped)
        rseed = 900 + it
        torch.manual_seed(rseed)
        rgb, _, mask, _, _, _ = render(gen, H, H, cam, focal, None, None, z_ * gain, S)
        torch.manual_seed(rseed)
        u_c.append(torch.rand(b, H, H, S))
        u_f.append(torch.rand(b * H * H, S))
        loss = F.l1_loss(rgb, target) * b
        loss.backward()
        opt.step()
        opt.zero_grad()
        R_.data[:] = F.normalize(R_.data, dim=-1)
        z0_.data.clamp_(-4, 4)
        s_.data.abs_()
        losses.append(float(loss))
        masks.append(float(mask.mean()))
    np.savez_compressed(os.path.join(OUT, 'inversion.npz'),
                        w_init=w_init.numpy(), cam0=cam0.numpy(), focal0=focal0.numpy(),
                        target=target.numpy(), u_coarse=torch.stack(u_c).numpy(),
                        u_fine=torch.stack(u_f).numpy(), losses=np.array(losses),
                        ws=(z_.detach() * gain).numpy(), z0=z0_.detach().numpy(),
                        t2=t2_.detach().numpy(), s=s_.detach().numpy(), q=R_.detach().numpy(),
                        meta_seed=np.array(seed), meta_H=np.array(H), meta_S=np.array(S),
                        meta_steps=np.array(steps), meta_scene_range=np.array(scene_range),
                        meta_sdf_shift=np.array(SDF_SHIFT), meta_flipped=np.array(int(flipped)))
    print('inversion losses', losses, 'mask', masks)


def zbuffer_cases():
    """The perspective eval scripts' render copy (eval_nusc_persp.py:43-231): z-buffer depth."""
    render_case('zbuffer', 10, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True, render_file='eval_nusc_persp.py')


def field_variant_cases():
    """The reference's other field heads (generator.py:637-641, 665-666): colour by
    wide_sigmoid_rescaled of 3 decoder features (--attention_values 0), standard NeRF density
    softplus(d - 1) (use_sdf False), and both."""
    render_case('rgbhead', 7, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True, attention_values=0)
    # --attention_values N < 10 (generator.py:363-402, 665-679 allow any N; nfi pads to its 10)
    render_case('attn5', 12, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True, attention_values=5)
    render_case('nerfdensity', 8, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=True,
                flipped=True, randomize=True, use_sdf=False)
    render_case('nerf_rgbhead', 9, b=1, H=8, W=8, S=8, R=12, scene_range=0.55, white_bg=False,
                flipped=False, randomize=False, attention_values=0, use_sdf=False)


def viewdir_cases():
    """--use_viewdir (generator.py:189-252, 376-377, 464-465, 661-663; run.py:216-219): the
    decoder's 32 features pass through the view-direction mapper closure; attention colour head
    (pose gradients flow through the mapper) and the wide-sigmoid head with a white background."""
    render_case('viewdir', 11, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True, use_viewdir=True)
    render_case('viewdir_rgbhead', 12, b=1, H=8, W=8, S=8, R=12, scene_range=0.55, white_bg=True,
                flipped=False, randomize=False, attention_values=0, use_viewdir=True)


def near_far_clamp_cases():
    """near/far clamps (nerf_utils.py:264-270): a camera inside the box, one facing away from it."""
    render_case('inside', 7, b=2, H=12, W=12, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True, inside=True)


SDF_SHIFT = 0.0


if __name__ == '__main__':
    torch.set_num_threads(4)
    if len(sys.argv) > 1:              # regenerate selected groups only
        for a in sys.argv[1:]:
            globals()[a]()
        sys.exit(0)
    producer_case()
    pose_cases()
    inversion_case()
    augment_cases()
    metrics_cases()
    stage_cases()
    seam_cases()
    # p3d_car-like: perspective, flipped, black bg, pose grads, random sampling
    render_case('p3d', 0, b=2, H=16, W=16, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, randomize=True)
    # shapenet-like: white bg, pose frozen (loaders.py:123), deterministic sampling
    render_case('shapenet', 1, b=2, H=12, W=12, S=8, R=16, scene_range=0.55, white_bg=True,
                flipped=False, randomize=False, force_no_cam_grad=True)
    # cub-like: ortho camera with bbox (nerf_utils.py:67-91)
    render_case('cub', 2, b=1, H=8, W=8, S=8, R=12, scene_range=2.0, white_bg=False,
                flipped=True, randomize=True, ortho=True, with_bbox=True)
    # perspective with bbox + center (nerf_utils.py:43-56; eval_*_persp.py callers)
    render_case('persp_center_bbox', 3, b=2, H=8, W=12, S=8, R=8, scene_range=1.4,
                white_bg=False, flipped=True, randomize=True, with_bbox=True, with_center=True)
    near_far_clamp_cases()
    field_variant_cases()
    viewdir_cases()
    zbuffer_cases()
    # eval outputs: normals + semantics; white background; coords
    extras_case('extras_ns', 4, b=2, H=8, W=8, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, compute_normals=True, compute_semantics=True, compute_coords=False)
    extras_case('extras_nw', 5, b=1, H=8, W=8, S=8, R=12, scene_range=0.55, white_bg=True,
                flipped=False, compute_normals=True, compute_semantics=False, compute_coords=False)
    extras_case('extras_coords', 6, b=1, H=8, W=8, S=8, R=12, scene_range=1.4, white_bg=False,
                flipped=True, compute_normals=False, compute_semantics=True, compute_coords=True)
