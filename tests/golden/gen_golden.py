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
  * per-stage nerf_utils functions (compute_near_far_planes, sample_pdf, get_ray_bundle).
Random draws of the reference (torch.rand_like / torch.rand) are recovered by re-seeding and
drawing the same shapes in the same order, and stored as `u_coarse` / `u_fine`.
"""

import ast
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


def extract_render(args_ns, dataset_config):
    src = open(os.path.join(REF, 'run.py')).read()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'render'][0]
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {'torch': torch, 'F': F, 'nerf_utils': nerf_utils, 'args': args_ns,
          'dataset_config': dataset_config}
    exec(compile(mod, os.path.join(REF, 'run.py'), 'exec'), ns)
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
                force_no_cam_grad=False, ortho=False, with_bbox=False, with_center=False):
    torch.manual_seed(1000 + seed)
    gen = generator.Generator(512, scene_range, attention_values=10, use_sdf=True,
                              disable_stylegan_noise=True)
    gen.eval()
    with torch.no_grad():
        gen.decoder.net[2].bias[0] -= 0.97     # mask mean ~0.6 instead of ~5e-4
        gen.beta.fill_(0.1)
        gen.alpha.fill_(1.0)
    planes = (1.87 * torch.randn(b, 3, 32, R, R)).requires_grad_()
    gen.synthesis_network = PlanesLeaf(planes)
    palette = generator.wide_sigmoid_rescaled(torch.randn(b, 10, 3)).detach().requires_grad_()
    cam, focal = make_cameras(b, scene_range, flipped, seed, ortho=ortho)
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
    args_ns = types.SimpleNamespace(use_viewdir=False, fine_sampling=True, use_sdf=True,
                                    attention_values=10)
    dataset_config = {'scene_range': scene_range, 'white_background': white_bg}
    render = extract_render(args_ns, dataset_config)

    rseed = 77 + seed
    torch.manual_seed(rseed)
    rgb, depth, mask, _, _, _ = render(gen, H, W, cam, focal, center, bbox, ws, S,
                                       randomize=randomize,
                                       extra_model_inputs={'attention_values': palette},
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
        'b2': gen.decoder.net[2].bias.detach(), 'palette': palette.detach(),
        'alpha': gen.alpha.detach(), 'beta': gen.beta.detach(),
        'cam': cam.detach(), 'u_coarse': u_coarse, 'u_fine': u_fine,
        'g_rgb': g_rgb, 'g_mask': g_mask,
        'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach(),
        'd_planes': planes.grad, 'd_palette': palette.grad,
    }
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
                ortho=int(ortho))
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


if __name__ == '__main__':
    torch.set_num_threads(4)
    stage_cases()
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
    # eval outputs: normals + semantics; white background; coords
    extras_case('extras_ns', 4, b=2, H=8, W=8, S=16, R=16, scene_range=1.4, white_bg=False,
                flipped=True, compute_normals=True, compute_semantics=True, compute_coords=False)
    extras_case('extras_nw', 5, b=1, H=8, W=8, S=8, R=12, scene_range=0.55, white_bg=True,
                flipped=False, compute_normals=True, compute_semantics=False, compute_coords=False)
    extras_case('extras_coords', 6, b=1, H=8, W=8, S=8, R=12, scene_range=1.4, white_bg=False,
                flipped=True, compute_normals=False, compute_semantics=True, compute_coords=True)
