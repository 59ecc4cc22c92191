"""The inversion loop around the renderer: run.py:1960-2310 for one batch of
target images — latent + pose optimised by Adam against an image loss, with the volume render
on the HIP path (nfi.render) and the producer (synthesis network + AttentionMapper) in
PyTorch-ROCm.

Pose representation (lib/pose_utils.py:48-128): `(z0, t2, s, q)` with focal f = 1 + exp(z0),
translation t3 = (t2/s, f/s) in camera space, rotation from the unit quaternion q;
`pose_to_matrix` / `matrix_to_pose` restate it in torch (the quaternion extraction is
Shepperd's method, as in the reference's `matrix_to_quaternion`).
"""

from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch
import torch.nn.functional as F

from . import producer_ops
from .render import render as _nfi_render


# ---------------------------------------------------------------------------------------------
# pose parameterisation (lib/pose_utils.py)

_CONST: dict = {}


def _const(name: str, dev, dtype, build):
    """Small constant tensors of the pose math, built once per (device, dtype): no host copy
    inside a step (a captured graph forbids one, and a pageable copy drains the launch queue)."""
    key = (name, dev, dtype)
    t = _CONST.get(key)
    if t is None:
        t = _CONST[key] = build().to(device=dev, dtype=dtype)
    return t


def _quat_table():
    """[16, 9]: the reference's rotation entries (pose_utils.py:41-45, row-major, before the
    transpose) as combinations of the products q_i q_j, (w, x, y, z) = 0..3; entry k =
    [1, 0, 0, 0, 1, 0, 0, 0, 1][k] + sum_ij q_i q_j T[4i + j, k]."""
    W, X, Y, Z = range(4)
    terms = [[(-2, Y, Y), (-2, Z, Z)], [(2, X, Y), (-2, W, Z)], [(2, X, Z), (2, W, Y)],
             [(2, X, Y), (2, W, Z)], [(-2, X, X), (-2, Z, Z)], [(2, Y, Z), (-2, W, X)],
             [(2, X, Z), (-2, W, Y)], [(2, Y, Z), (2, W, X)], [(-2, X, X), (-2, Y, Y)]]
    T = torch.zeros(16, 9, dtype=torch.float64)
    for k, ts in enumerate(terms):
        for c, i, j in ts:
            T[4 * i + j, k] += c
    return T


def quaternion_to_matrix(q: torch.Tensor) -> torch.Tensor:
    """pose_utils.py:41-45: the matrix whose rows are the unit vectors rotated by q, i.e. the
    transpose of the rotation matrix of q = (w, x, y, z).  Its entries are 1 or 0 plus quadratic
    forms in q: one outer product and one contraction with a constant table (4 kernels forward and
    backward instead of ~40 scalar-sized ones)."""
    T = _const('quat', q.device, q.dtype, _quat_table)
    eye = _const('eye9', q.device, q.dtype, lambda: torch.eye(3, dtype=torch.float64).reshape(9))
    qq = (q.unsqueeze(-1) * q.unsqueeze(-2)).reshape(q.shape[:-1] + (16, 1))
    r = (qq * T).sum(-2) + eye
    return r.view(q.shape[:-1] + (3, 3)).transpose(-2, -1)


def _flip(mat: torch.Tensor, camera_flipped: bool) -> torch.Tensor:
    """pose_utils.py:61: columns 1..3 of rows 0..2 negated."""
    if not camera_flipped:
        return mat
    sign = _const('flip', mat.device, mat.dtype,
                  lambda: torch.tensor([[1.0, -1.0, -1.0, -1.0]] * 3 + [[1.0, 1.0, 1.0, 1.0]]))
    return mat * sign


def pose_to_matrix(z0, t2, s, q, camera_flipped: bool):
    """pose_utils.py:48-78 -> (cam2world [b,4,4], focal or None)."""
    rot = quaternion_to_matrix(q)
    b = q.shape[0]
    if z0 is not None:
        f = 1 + z0.exp()
        t3 = torch.cat([t2, f[:, None]], dim=-1) / s[:, None]    # (t2 / s, f / s): same divisions
        focal = f / 2
    else:
        t3 = torch.cat([t2, torch.ones_like(t2[:, :1])], dim=-1) / s[:, None]
        focal = None
    top = torch.cat([rot, (rot * t3[:, None, :]).sum(-1, keepdim=True)], dim=-1)
    bottom = _const('bottom', top.device, top.dtype, lambda: torch.tensor([[[0.0, 0.0, 0.0, 1.0]]]))
    return _flip(torch.cat([top, bottom.expand(b, 1, 4)], dim=1), camera_flipped), focal


class _PoseHIP(torch.autograd.Function):
    """pose_to_matrix(z0, t2, s, F.normalize(q)) on device tensors as one HIP launch each way
    (nfi_pose_forward / nfi_pose_backward: the ~35 scalar-sized ATen kernels of the torch form)."""

    @staticmethod
    def forward(ctx, z0, t2, s, q, flipped: bool):
        from . import _lib
        from .ops import _ptr, _stream
        b = q.shape[0]
        z0c, t2c, sc, qc = (None if z0 is None else z0.contiguous()), t2.contiguous(), s.contiguous(), q.contiguous()
        cam = torch.empty((b, 4, 4), device=q.device)
        focal = torch.empty((b,), device=q.device) if z0 is not None else None
        _lib.check(_lib.load().nfi_pose_forward(_ptr(z0c), _ptr(t2c), _ptr(sc), _ptr(qc), b, int(flipped), _ptr(cam),
                                                _ptr(focal), _stream(q.device)), 'nfi_pose_forward')
        ctx.save_for_backward(*(t for t in (z0c, t2c, sc, qc) if t is not None))
        ctx.has_z0, ctx.flipped = z0 is not None, flipped
        return cam, focal

    @staticmethod
    def backward(ctx, g_cam, g_focal):
        from . import _lib
        from .ops import _ptr, _stream
        saved = ctx.saved_tensors
        z0, t2, s, q = saved if ctx.has_z0 else (None,) + tuple(saved)
        b = q.shape[0]
        g_cam = torch.zeros((b, 4, 4), device=q.device) if g_cam is None else g_cam.contiguous()
        d_z0 = torch.empty_like(z0) if z0 is not None else None
        d_t2, d_s, d_q = torch.empty_like(t2), torch.empty_like(s), torch.empty_like(q)
        _lib.check(_lib.load().nfi_pose_backward(
            _ptr(z0), _ptr(t2), _ptr(s), _ptr(q), b, int(ctx.flipped), _ptr(g_cam),
            _ptr(None if g_focal is None else g_focal.contiguous()), _ptr(d_z0), _ptr(d_t2), _ptr(d_s), _ptr(d_q),
            _stream(q.device)), 'nfi_pose_backward')
        return d_z0, d_t2, d_s, d_q, None


def pose_matrix(z0, t2, s, q, camera_flipped: bool):
    """pose_to_matrix(z0, t2, s, F.normalize(q, dim=-1), camera_flipped) (run.py:2262): the HIP
    kernels for device tensors, the torch formulation on the CPU."""
    if q.is_cuda:
        return _PoseHIP.apply(z0, t2, s, q, camera_flipped)
    return pose_to_matrix(z0, t2, s, F.normalize(q, dim=-1), camera_flipped)


def project_pose(z0, s, q):
    """The post-step projections (run.py:2300-2306), in place, no grad: q <- F.normalize(q),
    z0 <- clamp(z0, -4, 4), s <- |s|."""
    with torch.no_grad():
        if q.is_cuda:
            from . import _lib
            from .ops import _ptr, _stream
            _lib.check(_lib.load().nfi_pose_project(_ptr(z0), _ptr(s), _ptr(q), q.shape[0], _stream(q.device)),
                       'nfi_pose_project')
            for t in (z0, s, q):       # written in place behind autograd's back: mark them modified
                if t is not None:
                    torch.autograd.graph.increment_version(t)
            return
        q.copy_(F.normalize(q, dim=-1))
        if z0 is not None:
            z0.clamp_(-4, 4)
        s.abs_()


def invert_space(mat: torch.Tensor) -> torch.Tensor:
    """pose_utils.py:20-27: cam2world <-> world2cam of a scaled rigid transform."""
    scale = mat[:, 3:4, 3:4]
    rot = mat[:, :3, :3] / scale
    out = torch.zeros_like(mat)
    out[:, :3, :3] = rot.transpose(-2, -1)
    out[:, :3, 3] = -(rot * mat[:, :3, None, 3]).sum(-2)
    out[:, 3, 3].fill_(1.0)
    return out


def rotation_to_quaternion(m: torch.Tensor) -> torch.Tensor:
    """Shepperd's method on the 3x3 block of [b,4,4] matrices (pose_utils.py:81-100), float64;
    q = (w, x, y, z) with the sign fixed by the dominant component being positive."""
    m = m.double()
    hom = m[:, 3, 3]
    tr = m[:, 0, 0] + m[:, 1, 1] + m[:, 2, 2] + hom
    out = torch.empty(m.shape[0], 4, dtype=torch.float64, device=m.device)
    for n in range(m.shape[0]):
        M = m[n]
        t = float(tr[n])
        if t > float(hom[n]):
            q = [t, float(M[2, 1] - M[1, 2]), float(M[0, 2] - M[2, 0]), float(M[1, 0] - M[0, 1])]
        else:
            d = [float(M[0, 0]), float(M[1, 1]), float(M[2, 2])]
            i = 0
            if d[1] > d[0]:
                i = 1
            if d[2] > d[i]:
                i = 2
            j, k = (i + 1) % 3, (i + 2) % 3
            t = d[i] - (d[j] + d[k]) + float(hom[n])
            v = [0.0, 0.0, 0.0]
            v[i] = t
            v[j] = float(M[i, j] + M[j, i])
            v[k] = float(M[k, i] + M[i, k])
            q = [float(M[k, j] - M[j, k])] + v
        scale = 0.5 / math.sqrt(t * float(hom[n]))
        out[n] = torch.tensor(q, dtype=torch.float64) * scale
    return out


def matrix_to_pose(cam2world: torch.Tensor, focal: Optional[torch.Tensor], camera_flipped: bool):
    """pose_utils.py:103-128 -> (z0 or None, t2, s, q) (all detached, float32)."""
    mat = _flip(cam2world.detach(), camera_flipped)
    inv = invert_space(mat)
    t3 = -inv[:, :3, 3]
    if focal is not None:
        focal = focal.detach()
        z0 = torch.log(2 * focal - 1)
        s = 2 * focal / t3[:, 2]
    else:
        z0 = None
        s = 1 / t3[:, 2]
    t2 = t3[:, :2] * s[:, None]
    q = rotation_to_quaternion(inv.cpu()).float().to(t3.device)
    return z0, t2, s, q


# ---------------------------------------------------------------------------------------------
# the loop (run.py:1960-2310)

@dataclass
class InversionConfig:
    steps: int = 30                      # max(checkpoint_steps)
    lr: float = 2e-3                     # run.py:2007
    betas: tuple = (0.9, 0.95)
    gain_z: float = 5.0                  # --inv_gain_z (lr_gain_z, run.py:1749)
    loss: str = 'l1'                     # --inv_loss: 'vgg' (reference default) | 'vgg_nocrop' | 'mixed' | 'l1' | 'mse'
    white_background: bool = False       # dataset_config['white_background'] (augmentation fill)
    samples: int = 64                    # depth_samples_per_ray (fine sampling doubles it)
    resolution: int = 128
    optimize_pose: bool = True           # not --inv_no_optimize_pose
    no_split: bool = False               # --inv_no_split: one w shared by the 15 slots
    camera_flipped: bool = True          # dataset_config['camera_flipped']
    overlap_target: bool = True          # 'vgg' losses: target features on a side stream (GPU)
    graph: bool = False                  # GPU: replay the step as a captured HIP graph (see invert;
                                         # measured slower than eager launches on ROCm 7.2)
    adam: str = 'fused'                  # GPU Adam kernel: 'fused' (one kernel for all parameters) or
                                         # 'foreach' (torch's default on CUDA, the reference's run.py:2007):
                                         # the same update formula, rounded differently at ulp level
                                         # (tests/test_gpu_inversion.py bounds the trajectories' distance)


@dataclass
class InversionResult:
    ws: torch.Tensor                     # [b,15,512] (z_ * gain)
    z0: Optional[torch.Tensor]
    t2: torch.Tensor
    s: torch.Tensor
    q: torch.Tensor
    losses: list = field(default_factory=list)
    seconds: float = 0.0


def augment_grid(shape, p: float, dev, disable_scale: bool = False,
                 generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """The sampling grid of augment_impl (run.py:720-767) for images of `shape` [bs,C,H,W]: random
    rotation, scale and translation per image with probability p, as affine_grid(align_corners=
    False).  Random draws in the reference's order, on `dev` (or from `generator`)."""
    bs = shape[0]

    def rand(*sh):
        return torch.rand(sh, device=dev, generator=generator)

    def randn(*sh):
        return torch.randn(sh, device=dev, generator=generator)

    rot = (rand(bs) - 0.5) * 2 * math.pi
    rot = rot * (rand(bs) < p).float()
    if disable_scale:
        scale = torch.ones((bs,), device=dev)
    else:
        scale = torch.exp2(randn(bs) * 0.2)
        scale = torch.lerp(torch.ones_like(scale), scale, (rand(bs) < p).float())
    translation = randn(bs, 2) * 0.1
    translation = torch.lerp(torch.zeros_like(translation), translation, (rand(bs, 1) < p).float())
    c, s = torch.cos(rot), torch.sin(rot)
    rotm = torch.stack([torch.stack([c, -s], -1), torch.stack([s, c], -1)], 1)   # [bs,2,2]
    t = torch.stack([translation[:, 0], -translation[:, 1]], -1) * scale[:, None]
    theta = torch.cat([rotm * scale[:, None, None], (rotm * t[:, None, :]).sum(-1, keepdim=True)], -1)
    if theta.is_cuda and producer_ops.AFFINE_GRID_HIP:
        return producer_ops.affine_grid(theta, list(shape))
    return F.affine_grid(theta, list(shape), align_corners=False)


def apply_grid(img: torch.Tensor, grid: torch.Tensor, white_background: bool = False) -> torch.Tensor:
    """Bilinear grid_sample with zero padding (white for white-background datasets), run.py:754-764."""
    if white_background:
        img = img - 1
    out = F.grid_sample(img, grid, mode='bilinear', padding_mode='zeros', align_corners=False)
    return out + 1 if white_background else out


def augment_images(img: torch.Tensor, p: float, white_background: bool = False,
                   disable_scale: bool = False, generator: Optional[torch.Generator] = None):
    """augment_impl (run.py:720-767) for images only (pose None, as the loss calls it)."""
    grid = augment_grid(img.shape, p, img.device, disable_scale, generator)
    return apply_grid(img, grid, white_background)


VGG_LOSSES = ('vgg', 'vgg_nocrop', 'mixed')


def _copies(x):
    return x.unsqueeze(1).expand(-1, 15, -1, -1, -1).contiguous().flatten(0, 1)


def vgg_target(kind: str, target: torch.Tensor, lpips_net, white_background: bool = False,
               augment_generator=None):
    """The prediction-independent half of the 'vgg' losses: the augmentation grid (run.py:720-767
    draws, in the reference's order) and the LPIPS features of the target and its 15 augmented
    copies (no gradient).  Returns (grid or None, target features)."""
    tgt = target.permute(0, 3, 1, 2)
    if kind == 'vgg_nocrop':
        return None, lpips_net.target_features(tgt)
    b = tgt.shape[0]
    grid = augment_grid((15 * b, 6) + tuple(tgt.shape[2:]), 1.0, tgt.device, generator=augment_generator)
    with torch.no_grad():
        if target.is_cuda:
            aug_tgt = producer_ops.aug_sample(target[..., :3], grid, 15, white_background)
        else:
            aug_tgt = apply_grid(_copies(tgt), grid, white_background)
    return grid, lpips_net.target_features(torch.cat((tgt, aug_tgt), dim=0))


def image_loss(kind: str, rgb: torch.Tensor, target: torch.Tensor, lpips_net=None,
               white_background: bool = False, augment_generator=None, prepared=None) -> torch.Tensor:
    """optimize_iter (run.py:2205-2252): per-batch-summed image loss.  'vgg' = LPIPS over the
    image plus 15 augmented copies of (prediction, target) pairs; 'vgg_nocrop' without the
    copies; 'mixed' = ('vgg' + 'l1') / 2; 'l1'; 'mse'.  `prepared` = vgg_target(...) computed
    beforehand (the grid and the target's features; the loss then only runs the prediction)."""
    b = rgb.shape[0]
    if kind not in VGG_LOSSES + ('l1', 'mse'):
        raise NotImplementedError(f'inversion loss {kind!r}')
    if kind == 'mse':
        return F.mse_loss(rgb, target) * b
    loss = 0.
    if kind in VGG_LOSSES:
        if lpips_net is None:
            raise ValueError(f'inversion loss {kind!r} needs an LPIPS network (nfi.lpips.LPIPS with '
                             f'weights loaded via load_weights; none ship offline)')
        # the reference augments cat((pred, target), channels) expanded to 15 copies; grid_sample
        # treats channels independently, so the prediction and target copies are sampled with the
        # same grid separately (identical values), and only the prediction's copies carry a
        # gradient (the reference backpropagates into the target copies and drops the result at
        # the target leaf)
        grid, f1 = prepared if prepared is not None else vgg_target(kind, target, lpips_net,
                                                                     white_background, augment_generator)
        pred = rgb.permute(0, 3, 1, 2)
        if kind != 'vgg_nocrop':
            aug = (producer_ops.aug_sample(rgb, grid, 15, white_background) if rgb.is_cuda
                   else apply_grid(_copies(pred), grid, white_background))
            pred = torch.cat((pred, aug), dim=0)
        loss = loss + lpips_net(pred, f1=f1).mean() * b
    if kind in ('l1', 'mixed'):
        loss = loss + F.l1_loss(rgb, target) * b
    if kind == 'mixed':
        loss = loss / 2
    return loss


def invert(generator, target_img: torch.Tensor, cam2world: torch.Tensor, focal: Optional[torch.Tensor],
           w_init: torch.Tensor, cfg: InversionConfig = InversionConfig(), center=None, bbox=None,
           uniforms: Optional[Callable[[int], tuple]] = None, render_fn: Optional[Callable] = None,
           on_step: Optional[Callable] = None, lpips_net=None, checkpoints=(),
           on_checkpoint: Optional[Callable] = None) -> InversionResult:
    """Fit latent + pose of `generator` (frozen) to `target_img` [b,H,W,3 or 4] in [-1,1].

    `w_init` [1 or b, 15, 512] is the starting latent (z_avg or a regressor output);
    `cam2world`/`focal` the initial pose.  `lpips_net` (nfi.lpips.LPIPS) is needed by the
    'vgg' losses.  `uniforms(it) -> (u_coarse, u_fine)` fixes the
    renderer's random draws per iteration (parity tests); `render_fn` replaces nfi.render with
    a callable of the same signature (tests only).  `on_checkpoint(it, (z_, z0_, t2_, s_, q_))`
    runs before the first step if 0 is in `checkpoints` and after step it if it is
    (evaluate_inversion, run.py:2020-2110 and 2302-2305; see nfi.report.evaluate).

    On a HIP device with cfg.graph (and no injected draws / render_fn), the whole step — producer,
    render, loss, backward, Adam, the post-step projections — is captured once as a HIP graph
    (torch.cuda.CUDAGraph over the ROCm runtime) after two eager steps, and replayed: ~900
    kernel launches per step become one graph launch.  Measured on MI355X (B=4, 30 steps): L1
    step 13.2 ms eager vs 14.1 ms replayed, vgg 24.6 vs 25.6 ms — the replay of ~900 nodes costs
    more GPU time than it saves host time (the eager loop keeps the queue full), and the vgg
    loss's side stream no longer overlaps — so it is off by default.  The graph and its static tensors (latent,
    pose, Adam moments, target) are kept per (generator, loss network, shapes, config) and reused
    by later batches of the same shape, as the reference's loop over dataset batches
    (run.py:1874) would; each batch copies its inputs into them and resets Adam.  The renderer's
    stratified / inverse-CDF draws then come from torch's device generator (graph-safe) instead
    of the kernels' host-seeded Philox stream: same distribution, another stream."""
    use_graph = (cfg.graph and target_img.is_cuda and uniforms is None and render_fn is None)
    if use_graph:
        return _invert_graphed(generator, target_img, cam2world, focal, w_init, cfg, center, bbox,
                               on_step, lpips_net, checkpoints, on_checkpoint)
    b = target_img.shape[0]
    rfn = render_fn or _nfi_render
    st = _State(generator, target_img, cam2world, focal, w_init, cfg, center, bbox, lpips_net,
                capturable=False)
    losses = []
    if on_checkpoint is not None and 0 in checkpoints:
        on_checkpoint(0, st.views())
    t0 = time.perf_counter()
    for it in range(cfg.steps):
        kw = {}
        if uniforms is not None:
            kw['u_coarse'], kw['u_fine'] = uniforms(it)
        loss = st.step(rfn, kw)
        losses.append(loss.detach())
        if on_step is not None:
            on_step(it, loss)
        if on_checkpoint is not None and it + 1 in checkpoints:
            on_checkpoint(it + 1, st.views())
    if torch.cuda.is_available() and target_img.is_cuda:
        torch.cuda.synchronize(target_img.device)
    secs = time.perf_counter() - t0
    assert b == st.b
    return st.result(losses, secs)


class _State:
    """The optimised tensors of one inversion batch (run.py:1984-2007) and one step of the loop
    (run.py:2256-2310) over them."""

    def __init__(self, generator, target_img, cam2world, focal, w_init, cfg, center, bbox, lpips_net,
                 capturable: bool):
        self.gen, self.cfg, self.lpips_net = generator, cfg, lpips_net
        self.b = target_img.shape[0]
        z_ = w_init.detach().clone().expand(self.b, -1, -1).contiguous()
        if cfg.no_split:
            z_ = z_.mean(dim=1, keepdim=True)
        self.z_ = (z_ / cfg.gain_z).requires_grad_()
        self.z0_, self.t2_, self.s_, self.q_ = matrix_to_pose(cam2world, focal, cfg.camera_flipped)
        params = [self.z_]
        if cfg.optimize_pose:
            pose = [p for p in (self.z0_, self.q_, self.s_, self.t2_) if p is not None]
            for p in pose:
                p.requires_grad_()
            params += pose
        self.params = params
        # on the GPU the fused Adam by default: one kernel for the latent and the pose tensors instead of
        # the foreach form's per-op launches (same update formula as run.py:2007's default Adam, rounded
        # differently: cfg.adam = 'foreach' selects the reference's form for parity runs)
        if cfg.adam not in ('fused', 'foreach'):
            raise ValueError(f"InversionConfig.adam must be 'fused' or 'foreach', not {cfg.adam!r}")
        fused = bool(params[0].is_cuda) and cfg.adam == 'fused'
        self.opt = torch.optim.Adam(params, lr=cfg.lr, betas=cfg.betas, capturable=capturable,
                                    **({'fused': True} if fused else {}))
        self.target = target_img[..., :3]
        if capturable:
            # a private static buffer: later batches are copied into it (load), which must never
            # overwrite the caller's first target image
            self.target = self.target.clone(memory_format=torch.contiguous_format)
        self.center, self.bbox = center, bbox
        # the prediction-independent half of the 'vgg' losses (augmentation grid, LPIPS features
        # of the target and its copies) runs on a side stream, concurrently with the producer and
        # the render
        self.side = None
        if cfg.loss in VGG_LOSSES and self.target.is_cuda and cfg.overlap_target:
            self.side = torch.cuda.Stream(device=self.target.device)

    def views(self):
        return self.z_, self.z0_, self.t2_, self.s_, self.q_

    def load(self, target_img, cam2world, focal, w_init, center, bbox):
        """A new batch into the same (static) tensors; Adam restarts (run.py:2007 builds a new
        optimiser per batch)."""
        cfg = self.cfg
        with torch.no_grad():
            z_ = w_init.detach().expand(self.b, -1, -1)
            if cfg.no_split:
                z_ = z_.mean(dim=1, keepdim=True)
            self.z_.copy_(z_ / cfg.gain_z)
            z0, t2, s, q = matrix_to_pose(cam2world, focal, cfg.camera_flipped)
            for dst, src in ((self.z0_, z0), (self.t2_, t2), (self.s_, s), (self.q_, q)):
                if dst is not None:
                    dst.copy_(src)
            self.target.copy_(target_img[..., :3])
            for dst, src in ((self.center, center), (self.bbox, bbox)):
                if dst is not None:
                    dst.copy_(src)
            for p in self.params:
                state = self.opt.state.get(p)
                if state:
                    state['step'].zero_()
                    state['exp_avg'].zero_()
                    state['exp_avg_sq'].zero_()

    def step(self, rfn, kw):
        """One step (run.py:2256-2310): producer + render, loss, backward, Adam, projections.
        Returns the loss (the per-batch sum, as the reference's `loss.sum()`)."""
        cfg = self.cfg
        prepared = None
        side = self.side
        if side is not None:
            main = torch.cuda.current_stream(self.target.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                prepared = vgg_target(cfg.loss, self.target, self.lpips_net, cfg.white_background)
        cam, foc = pose_matrix(self.z0_, self.t2_, self.s_, self.q_, cfg.camera_flipped)
        ws = self.z_ * cfg.gain_z
        if cfg.no_split:
            ws = ws.expand(-1, 15, -1)
        rgb = rfn(self.gen, cfg.resolution, cfg.resolution, cam, foc, self.center, self.bbox, ws, cfg.samples,
                  force_no_cam_grad=not cfg.optimize_pose, **kw)[0]
        if side is not None:
            main.wait_stream(side)
            for t in ([prepared[0]] if prepared[0] is not None else []) + list(prepared[1]):
                t.record_stream(main)
        loss = image_loss(cfg.loss, rgb, self.target, self.lpips_net, cfg.white_background, prepared=prepared)
        loss.backward()
        self.opt.step()
        self.opt.zero_grad()
        project_pose(self.z0_, self.s_, self.q_)
        return loss

    def result(self, losses, secs):
        cfg = self.cfg
        ws = (self.z_.detach() * cfg.gain_z)
        if cfg.no_split:
            ws = ws.expand(-1, 15, -1)
        z0 = self.z0_
        return InversionResult(ws=ws.clone(), z0=None if z0 is None else z0.detach().clone(),
                               t2=self.t2_.detach().clone(), s=self.s_.detach().clone(),
                               q=self.q_.detach().clone(), losses=[float(x) for x in losses], seconds=secs)


_GRAPHS: dict = {}
EAGER_STEPS = 2           # eager steps before the capture (Adam state, frozen caches, library plans)


def _graph_key(generator, target_img, cam2world, focal, w_init, cfg, center, bbox, lpips_net):
    import dataclasses

    def shape(t):
        return None if t is None else (tuple(t.shape), t.dtype, t.device)
    return (id(generator), id(lpips_net), shape(target_img), shape(cam2world), shape(focal), shape(w_init),
            shape(center), shape(bbox), dataclasses.astuple(cfg))


def _invert_graphed(generator, target_img, cam2world, focal, w_init, cfg, center, bbox, on_step, lpips_net,
                    checkpoints, on_checkpoint):
    key = _graph_key(generator, target_img, cam2world, focal, w_init, cfg, center, bbox, lpips_net)
    entry = _GRAPHS.get(key)
    fresh = entry is None or entry['gen'] is not generator or entry['net'] is not lpips_net
    if fresh:
        cen = None if center is None else center.detach().clone()
        bb = None if bbox is None else bbox.detach().clone()
        st = _State(generator, target_img, cam2world, focal, w_init, cfg, cen, bb, lpips_net, capturable=True)
        entry = {'gen': generator, 'net': lpips_net, 'state': st, 'graph': None, 'loss': None}
        _GRAPHS.clear()              # one live graph (its memory pool) at a time
        _GRAPHS[key] = entry
    else:
        st = entry['state']
        st.load(target_img, cam2world, focal, w_init, center, bbox)
    dev = target_img.device
    losses = []
    if on_checkpoint is not None and 0 in checkpoints:
        on_checkpoint(0, st.views())
    t0 = time.perf_counter()
    loss = None
    for it in range(cfg.steps):
        if entry['graph'] is None and it == EAGER_STEPS and cfg.steps > EAGER_STEPS:
            # the capture records one step without running it; replays run it.  The eager steps'
            # autograd graphs must be gone first: a live one keeps the leaves' AccumulateGrad nodes
            # bound to the eager stream, and the capture would then wait on that stream
            loss = None
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                entry['loss'] = st.step(_nfi_render, {})
            entry['graph'] = g
        if entry['graph'] is not None:
            entry['graph'].replay()
            loss = entry['loss']
        else:
            # eager steps take the same device draws the graph does
            with _capturing_draws():
                loss = st.step(_nfi_render, {})
        losses.append(loss.detach().clone())
        if on_step is not None:
            on_step(it, loss)
        if on_checkpoint is not None and it + 1 in checkpoints:
            on_checkpoint(it + 1, st.views())
    torch.cuda.synchronize(dev)
    secs = time.perf_counter() - t0
    return st.result(losses, secs)


class _capturing_draws:
    """Eager steps of a graphed inversion draw the renderer's uniforms from torch's device
    generator too (ops.volume_render does so while a capture is running)."""

    def __enter__(self):
        from . import ops
        self.prev, ops.DEVICE_DRAWS = ops.DEVICE_DRAWS, True
        return self

    def __exit__(self, *exc):
        from . import ops
        ops.DEVICE_DRAWS = self.prev
        return False
