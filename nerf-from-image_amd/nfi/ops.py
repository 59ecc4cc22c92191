"""Autograd operators over the nfi C-ABI (HIP kernels).  Device tensors only — there is no
CPU path: every op raises if its inputs are not on a HIP device.

Operators (reference function each one replaces, file:line in yuliangguo/nerf-from-image):
  planes_texel_major   layout of generator.py:476-477 planes for the tap kernels
  rays                 nerf_utils.get_ray_bundle (:28-93) + F.normalize (run.py:196)
                       + nerf_utils.compute_near_far_planes (:227-275, no grad)
  volume_render        run.py:202-348 from the rays onward: compute_query_points_from_rays,
                       sampler (generator.py:587-681) coarse + fine, weights/smoothing,
                       sample_pdf, sort/merge, render_volume_density — fused
"""

from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib


def _ptr(t: Optional[torch.Tensor]):
    # (a plain int: the ctypes prototypes declare c_void_p, which converts it — no wrapper object)
    return None if t is None else t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream


def _stream(dev: torch.device):
    """The current HIP stream of dev as an int (the raw handle: no torch.cuda.Stream object per launch)."""
    return _raw_stream(dev.index if dev.index is not None else torch.cuda.current_device())


# Optional live kernel timing (bench.py): name -> list of (start, end) events recorded on the
# stream the C-ABI call launches on.  Off by default (no events, no overhead).
# The forward counts the backward's tile bins (nfi_render_args.tile_counts) when True; when
# False the backward counts them itself (both paths are covered by tests/test_gpu_parity.py).
FORWARD_TILE_COUNTS = True

# Bitwise-reproducible backward (nfi_set_deterministic): tile bins sorted by sample, d planes summed
# in a fixed order without float atomics.  None: follow torch.use_deterministic_algorithms() (and the
# NFI_DETERMINISTIC environment variable, read by the library); True / False: force.
DETERMINISTIC: Optional[bool] = None


def _deterministic() -> bool:
    if DETERMINISTIC is not None:
        return bool(DETERMINISTIC)
    return torch.are_deterministic_algorithms_enabled() or os.environ.get('NFI_DETERMINISTIC', '0') not in ('', '0')

KERNEL_TIMERS: Optional[dict] = None

# randomized renders draw their uniforms with torch.rand on the device (graph-safe) instead of the
# kernels' host-seeded Philox stream: always while a HIP graph is being captured, and when set
# (the eager steps of a graphed inversion, nfi.inversion)
DEVICE_DRAWS = False


class _timed:
    """HIP events around one C-ABI call, recorded on the stream it launches on."""

    def __init__(self, name, dev, stream=None):
        self.name, self.dev, self.stream = name, dev, stream

    def __enter__(self):
        self.on = KERNEL_TIMERS is not None and not torch.cuda.is_current_stream_capturing()
        if self.on:
            self.s = self.stream if self.stream is not None else torch.cuda.current_stream(self.dev)
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record(self.s)
        return self

    def __exit__(self, *exc):
        if self.on:
            self.e1.record(self.s)
            KERNEL_TIMERS.setdefault(self.name, []).append((self.e0, self.e1))
        return False


# Optional: the backward of a batch of >= 2 images in two image halves, the tile pass of the first
# half on a side stream beside the field backward of the second.  Measured slower on MI355X (p3d
# B=8: 7.49 vs 7.39 ms per step; the overlapped launches stretch to 2.61 / 3.39 ms from 2.27 /
# 2.25: the two compete for the memory pipeline, not for different units), so off by default.
BACKWARD_PIPELINE = os.environ.get('NFI_BACKWARD_PIPELINE', '0') == '1'
# Slabs (A/B knob): the backward of NFI_BACKWARD_SLAB images at a time — bins,
# field backward, tile pass — so a slab's gradient rows are read back by the tile pass while the
# Infinity Cache still holds them; 0 = the whole batch in one pass of each stage
BACKWARD_SLAB = int(os.environ.get('NFI_BACKWARD_SLAB', '0'))
_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return s


def _require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('nfi ops run on HIP devices only (got a CPU tensor); '
                               'the CPU path of the reference is not part of this package')
        if t is not None and t.dtype != torch.float32:
            raise RuntimeError(f'nfi ops need float32 tensors (got {t.dtype})')


# ----------------------------------------------------------------------------------------
# Plane layout
# ----------------------------------------------------------------------------------------

class _PlanesTexelMajor(torch.autograd.Function):
    @staticmethod
    def forward(ctx, planes):
        lib = _lib.load()
        B, three, C, R, R2 = planes.shape
        src = planes.contiguous()
        out = torch.empty((B, 3, R, R, C), device=planes.device, dtype=planes.dtype)
        _lib.check(lib.nfi_planes_to_texel_major(_ptr(src), B, R, _ptr(out), _stream(planes.device)),
                   'nfi_planes_to_texel_major')
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        g = g.contiguous()
        B, _, R, _, C = g.shape
        out = torch.empty((B, 3, C, R, R), device=g.device, dtype=g.dtype)
        _lib.check(lib.nfi_planes_to_channel_major(_ptr(g), B, R, _ptr(out), _stream(g.device)),
                   'nfi_planes_to_channel_major')
        return out


def planes_texel_major(planes: torch.Tensor) -> torch.Tensor:
    """[B,3,32,R,R] planes (generator.py:476-477) -> texel-major [B,3,R,R,32] view/copy.
    A channels_last producer output is re-viewed without a copy."""
    _require_device(planes)
    if planes.dim() != 5 or planes.shape[1] != 3 or planes.shape[2] != 32 or planes.shape[3] != planes.shape[4]:
        raise ValueError(f'planes must be [B,3,32,R,R], got {tuple(planes.shape)}')
    tm = planes.permute(0, 1, 3, 4, 2)
    # the view is used only when it is also dense (non-overlapping, no gaps): the backward writes
    # d planes with the view's strides into torch.zeros_like(view), which keeps the strides only
    # for dense tensors (a batch-sliced or channel-sliced channels_last buffer is copied instead)
    if tm.stride(-1) == 1 and tm.stride(2) == tm.shape[3] * tm.stride(3) and _dense(tm):
        return tm
    return _PlanesTexelMajor.apply(planes)


def _dense(t: torch.Tensor) -> bool:
    """True when t's elements tile its storage span exactly (torch's non-overlapping-and-dense)."""
    expected = 1
    for size, stride in sorted(((s, st) for s, st in zip(t.shape, t.stride()) if s != 1), key=lambda p: p[1]):
        if stride != expected:
            return False
        expected *= size
    return True


# ----------------------------------------------------------------------------------------
# Rays
# ----------------------------------------------------------------------------------------

def _camera_struct(cam, focal, center, bbox, H, W):
    return _lib.NfiCamera(cam=_ptr(cam), focal=_ptr(focal), center=_ptr(center), bbox=_ptr(bbox),
                          B=cam.shape[0], H=H, W=W, _pad=0)


class _Rays(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam, focal, center, bbox, H: int, W: int, scene_range: float):
        lib = _lib.load()
        B = cam.shape[0]
        dev = cam.device
        n = B * H * W
        cam_c = cam.contiguous()
        foc_c = None if focal is None else focal.contiguous()
        cen_c = None if center is None else center.contiguous()
        bb_c = None if bbox is None else bbox.contiguous()
        ro = torch.empty((B, H, W, 3), device=dev)
        rd = torch.empty((B, H, W, 3), device=dev)
        near = torch.empty((B, H, W), device=dev)
        far = torch.empty((B, H, W), device=dev)
        ws = torch.empty((2 + n,), device=dev, dtype=torch.int32)
        cs = _camera_struct(cam_c, foc_c, cen_c, bb_c, H, W)
        _lib.check(lib.nfi_rays_forward(ctypes.byref(cs), float(scene_range), _ptr(ro), _ptr(rd),
                                        _ptr(near), _ptr(far), _ptr(ws), _stream(dev)),
                   'nfi_rays_forward')
        ctx.save_for_backward(cam_c, foc_c, cen_c, bb_c)
        ctx.HW = (H, W)
        ctx.mark_non_differentiable(near, far)
        return ro, rd, near, far

    @staticmethod
    def backward(ctx, g_ro, g_rd, g_near, g_far):
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
        _lib.check(lib.nfi_rays_backward(ctypes.byref(cs), _ptr(g_ro), _ptr(g_rd), _ptr(contrib), st),
                   'nfi_rays_backward')
        red = torch.empty((B, 16), device=dev)
        ws = torch.empty((B * 64 * 16,), device=dev)
        _lib.check(lib.nfi_segment_sum(_ptr(contrib), B, H * W, 16, _ptr(red), _ptr(ws), st),
                   'nfi_segment_sum')
        d_cam = torch.zeros((B, 4, 4), device=dev)
        d_cam[:, :3, :] = red[:, :12].view(B, 3, 4)
        d_cam[:, 3, 3] = red[:, 12]
        d_focal = red[:, 13].clone() if focal is not None else None
        return d_cam, d_focal, None, None, None, None, None


def rays(cam, focal, center, bbox, H: int, W: int, scene_range: float):
    """get_ray_bundle + F.normalize + near/far (run.py:193-200) -> ro, rd [B,H,W,3], near, far."""
    _require_device(cam, focal, center, bbox)
    return _Rays.apply(cam, focal, center, bbox, int(H), int(W), float(scene_range))


# ----------------------------------------------------------------------------------------
# Fused volume render
# ----------------------------------------------------------------------------------------

@dataclass
class RenderOptions:
    samples: int                 # depth_samples_per_ray (coarse; fine adds as many)
    fine: bool = True            # args.fine_sampling
    white_background: bool = False
    randomize: bool = True
    scene_range: float = 1.0
    inv_alpha: float = 1.0       # 1 / Generator.alpha
    beta: float = 0.1            # Generator.beta
    extras: int = 0              # eval outputs: 1 normals, 2 semantics, 4 coords (nfi_render_args.extras)
    heads: int = 0               # nfi_field.heads: HEAD_RGB_SIGMOID (attention_values 0) | HEAD_NERF_DENSITY (no SDF)
                                 # | HEAD_VIEWDIR (view-direction mapper)


HEAD_RGB_SIGMOID = 1             # include/nfi.h NFI_HEAD_RGB_SIGMOID
DEBUG_BACKWARD = None            # a dict: the next backward stores its workspace there (diagnostics)
HEAD_NERF_DENSITY = 2            # include/nfi.h NFI_HEAD_NERF_DENSITY
HEAD_VIEWDIR = 4                 # include/nfi.h NFI_HEAD_VIEWDIR


def pack_decoder(w1, b1, w2, b2, lr_multiplier: float = 1.0, key_tensors=None) -> torch.Tensor:
    """EqualizedLinear gains (stylegan.py:173-176) folded into the packed decoder buffer.  A
    [4, 64] output layer (attention_values 0: distance + 3 colour features) is zero-padded to the
    kernels' 11 rows; a [33, 64] layer (the view-direction mapper's decoder, generator.py:376-377)
    is packed in its own layout (nfi_decoder_pack_n, nout 33).
    `key_tensors`: the caller's own (w1, b1, w2, b2) when w2 / b2 here are padded copies of them
    (render.attention_padded): the cache is keyed on the tensors whose in-place updates bump a version,
    never on a fresh copy whose storage the allocator may hand out again."""
    _require_device(w1, b1, w2, b2)
    nout = 33 if w2.shape[0] == 33 else 11
    # a pure function of the four tensors' values: cached on w1 per (storage, version) of the caller's
    # four tensors, taken before any padding — the inversion packs the same frozen decoder every step
    # (one kernel + host work saved per step)
    kt = tuple(key_tensors) if key_tensors is not None else (w1, b1, w2, b2)
    key = tuple((t.data_ptr(), t._version, tuple(t.shape)) for t in kt) + (float(lr_multiplier), w1.device)
    hit = getattr(w1, '_nfi_dec', None)
    if hit is not None and hit[0] == key:
        return hit[1]
    if w2.shape[0] < 11:
        w2 = torch.cat([w2.detach(), w2.new_zeros(11 - w2.shape[0], w2.shape[1])])
        b2 = torch.cat([b2.detach(), b2.new_zeros(11 - b2.shape[0])])
    if w2.shape[0] != nout:
        raise ValueError(f'decoder output layer must have <= 11 or 33 rows, got {w2.shape[0]}')
    lib = _lib.load()
    dec = torch.empty((int(lib.nfi_decoder_size(nout)),), device=w1.device)
    g1 = float(torch.tensor(lr_multiplier / math.sqrt(w1.shape[1]), dtype=torch.float32))
    g2 = float(torch.tensor(lr_multiplier / math.sqrt(w2.shape[1]), dtype=torch.float32))
    gb = float(torch.tensor(lr_multiplier, dtype=torch.float32))
    _lib.check(lib.nfi_decoder_pack_n(_ptr(w1.detach().contiguous()), _ptr(b1.detach().contiguous()),
                                      _ptr(w2.detach().contiguous()), _ptr(b2.detach().contiguous()), nout,
                                      g1, g2, gb, _ptr(dec), _stream(w1.device)), 'nfi_decoder_pack_n')
    try:
        w1._nfi_dec = (key, dec)
    except (AttributeError, RuntimeError):   # (a view or a tensor that takes no attributes: no cache)
        pass
    return dec


def pack_viewdir_head(weight, bias, lr_multiplier: float = 1.0) -> torch.Tensor:
    """ViewDirectionMapper.output (EqualizedLinear(32, O), generator.py:216-218) -> the kernels'
    vhead buffer: [O,32] gain-scaled weights then [O] scaled bias (nfi_field.vhead)."""
    _require_device(weight, bias)
    gain = float(torch.tensor(lr_multiplier / math.sqrt(weight.shape[1]), dtype=torch.float32))
    return torch.cat([(weight.detach() * gain).reshape(-1), (bias.detach() * lr_multiplier).reshape(-1)]).contiguous()


class _VolumeRender(torch.autograd.Function):
    @staticmethod
    def forward(ctx, planes_tm, palette, ro, rd, near, far, dec, opts: RenderOptions,
                u_coarse, u_fine, seed: int, debug: Optional[dict], xray=None, vhead=None):
        lib = _lib.load()
        B, _, R, R2, C = planes_tm.shape
        H, W = ro.shape[1], ro.shape[2]
        dev = ro.device
        n = B * H * W
        S = opts.samples
        N = 2 * S if opts.fine else S
        ro_c, rd_c = ro.contiguous(), rd.contiguous()
        near_c, far_c = near.contiguous(), far.contiguous()
        pal_c = None if palette is None else palette.contiguous()
        rgb = torch.empty((n, 3), device=dev)
        depth = torch.empty((n,), device=dev)
        mask = torch.empty((n,), device=dev)
        # per-sample state for the backward / eval outputs / debug; a forward-only call skips it
        keep = any(ctx.needs_input_grad) or bool(opts.extras) or debug is not None
        t_saved = torch.empty((n, N), device=dev) if keep else None
        s_saved = torch.empty((n, N), device=dev) if keep else None
        c_saved = torch.empty((n, 3, N), device=dev) if keep else None
        nout = 33 if opts.heads & HEAD_VIEWDIR else 11
        y_saved = torch.empty((n, nout, N), device=dev) if keep else None
        xray_c = None if xray is None else xray.contiguous()
        perm = torch.empty((n, N), device=dev, dtype=torch.int16) if keep else None
        # decoder inputs for the backward (saves it the re-gather) and for the normals pass
        need_x = any(ctx.needs_input_grad) or bool(opts.extras & 1)
        x_saved = torch.empty((n * N, 32), device=dev) if need_x else None
        nmap = torch.empty((n, 3), device=dev) if opts.extras & 1 else torch.empty(0, device=dev)
        smap = (torch.empty((n, 3 if opts.extras & 4 else 10), device=dev) if opts.extras & 6
                else torch.empty(0, device=dev))
        zc = zf = None
        if debug is not None:
            zc = torch.empty((n, S), device=dev)
            zf = torch.empty((n, S), device=dev) if opts.fine else None
        uc = None if u_coarse is None else u_coarse.contiguous()
        uf = None if u_fine is None else u_fine.contiguous()
        args = _VolumeRender._args(planes_tm, dec, pal_c, ro_c, rd_c, near_c, far_c, opts, B, H * W,
                                   uc, uf, seed, rgb, depth, mask, t_saved, s_saved, c_saved, y_saved, perm,
                                   zc, zf)
        args.x_saved = _ptr(x_saved)
        _VolumeRender._set_viewdir(args, opts, xray_c, vhead)
        args.extras = int(opts.extras)
        args.normal_map = _ptr(nmap) if nmap.numel() else None
        args.semantic_map = _ptr(smap) if smap.numel() else None
        tile_counts = None
        if FORWARD_TILE_COUNTS and ctx.needs_input_grad[0]:
            # the forward counts the backward's d-planes tile bins while it has the samples
            tile_counts = torch.empty((lib.nfi_tile_count_size(ctypes.byref(args)),), device=dev,
                                      dtype=torch.int32)
            args.tile_counts = _ptr(tile_counts)
        with _timed('render_fwd', dev):
            _lib.check(lib.nfi_render_forward(ctypes.byref(args), _stream(dev)), 'nfi_render_forward')
        if debug is not None:
            debug['z_coarse'] = zc
            debug['z_fine'] = zf
            debug['t_sorted'] = t_saved
            debug['sigma_sorted'] = s_saved
            debug['rgb_sorted'] = c_saved
            # the launch's argument block and the tensors it points at (scripts/gather_probe.py)
            debug['args'] = args
            debug['args_tensors'] = (planes_tm, pal_c, ro_c, rd_c, near_c, far_c, dec)
        ctx.save_for_backward(planes_tm, pal_c, ro_c, rd_c, near_c, far_c, dec, t_saved, s_saved, c_saved,
                              y_saved, perm, x_saved, tile_counts, xray_c, vhead)
        ctx.opts = opts
        ctx.shape = (B, H, W)
        ctx.mark_non_differentiable(depth, nmap, smap)
        if nmap.numel():
            nmap = nmap.view(B, H, W, 3)
        if smap.numel():
            smap = smap.view(B, H, W, -1)
        return rgb.view(B, H, W, 3), depth.view(B, H, W), mask.view(B, H, W), nmap, smap

    @staticmethod
    def _set_viewdir(args, opts, xray, vhead):
        if opts.heads & HEAD_VIEWDIR:
            if xray is None or vhead is None:
                raise ValueError('HEAD_VIEWDIR needs xray and vhead')
            args.field.xray = _ptr(xray)
            args.field.vhead = _ptr(vhead)
            args.field.vhead_out = 3 if opts.heads & HEAD_RGB_SIGMOID else 10

    @staticmethod
    def _args(planes_tm, dec, pal, ro, rd, near, far, opts, B, HW, uc, uf, seed, rgb, depth, mask,
              t_saved, s_saved, c_saved, y_saved, perm, zc, zf):
        W = ro.shape[2] if ro.dim() == 4 else 0
        R = planes_tm.shape[2]
        field = _lib.NfiField(planes=_ptr(planes_tm), sb=planes_tm.stride(0), sq=planes_tm.stride(1),
                              st=planes_tm.stride(3), R=R, _pad=0, dec=_ptr(dec), palette=_ptr(pal),
                              inv_alpha=float(opts.inv_alpha), beta=float(opts.beta),
                              scene_range=float(opts.scene_range), heads=int(opts.heads))
        return _lib.NfiRenderArgs(field=field, ro=_ptr(ro), rd=_ptr(rd), near_=_ptr(near), far_=_ptr(far),
                                  B=B, HW=HW, S=opts.samples, fine=int(opts.fine),
                                  white_bg=int(opts.white_background), randomize=int(opts.randomize),
                                  W=int(W),
                                  seed=seed & ((1 << 64) - 1), offset=0, u_coarse=_ptr(uc),
                                  u_fine=_ptr(uf), rgb=_ptr(rgb), depth=_ptr(depth), mask=_ptr(mask),
                                  t_saved=_ptr(t_saved), sigma_saved=_ptr(s_saved),
                                  rgb_saved=_ptr(c_saved), y_saved=_ptr(y_saved), perm=_ptr(perm),
                                  z_coarse=_ptr(zc), z_fine=_ptr(zf))

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_mask, g_nmap=None, g_smap=None):
        lib = _lib.load()
        planes_tm, pal, ro, rd, near, far, dec, t_saved, s_saved, c_saved, y_saved, perm, x_saved, \
            tile_counts, xray, vhead = ctx.saved_tensors
        opts = ctx.opts
        B, H, W = ctx.shape
        dev = ro.device
        n = B * H * W
        g_rgb = torch.zeros((n, 3), device=dev) if g_rgb is None else g_rgb.contiguous().view(n, 3)
        g_mask = torch.zeros((n,), device=dev) if g_mask is None else g_mask.contiguous().view(n)
        d_planes = torch.zeros_like(planes_tm)   # preserves (texel-major) strides: planes_tm is dense
        if d_planes.stride() != planes_tm.stride():
            raise RuntimeError(f'nfi: d planes strides {d_planes.stride()} differ from the planes view '
                               f'{planes_tm.stride()} (non-dense planes view)')
        npl = ((2 * opts.samples if opts.fine else opts.samples) + 63) // 64
        d_pal_ray = torch.empty((n * npl, 30), device=dev) if pal is not None else None
        need_coords = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        # per-(ray, chunk) partials of dL/d xray, summed over a ray's chunks below (fixed order)
        d_xray = torch.empty((n * npl, 32), device=dev) if xray is not None else None
        g_ro = torch.empty((n, 3), device=dev) if need_coords else None
        g_rd = torch.empty((n, 3), device=dev) if need_coords else None
        HW = H * W
        N = 2 * opts.samples if opts.fine else opts.samples
        per_img = None
        if tile_counts is not None:
            per_img = tile_counts.numel() // B
        # (per host thread: this is the thread running the backward — autograd's device thread for
        # .backward() — whatever the caller's thread set; restored below.  Workspace size and launches
        # follow it.)
        det = 1 if _deterministic() else 0
        prev_det = lib.nfi_set_deterministic(det)
        if DEBUG_BACKWARD is not None:
            DEBUG_BACKWARD['deterministic'] = int(lib.nfi_set_deterministic(-1))

        def part(b0, nb):
            """C-ABI arguments of the backward of images b0 .. b0+nb-1 (every per-image / per-ray
            buffer offset to the part; the d planes tile bins are keyed per image)."""
            r0, r1 = b0 * HW, (b0 + nb) * HW
            a = _VolumeRender._args(planes_tm[b0:b0 + nb], dec, None if pal is None else pal[b0:b0 + nb],
                                    ro[b0:b0 + nb], rd[b0:b0 + nb], near[b0:b0 + nb], far[b0:b0 + nb], opts, nb,
                                    HW, None, None, 0, None, None, None, t_saved[r0:r1], s_saved[r0:r1],
                                    c_saved[r0:r1], y_saved[r0:r1], perm[r0:r1], None, None)
            a.x_saved = _ptr(x_saved[r0 * N:r1 * N])
            _VolumeRender._set_viewdir(a, opts, None if xray is None else xray.view(n, -1)[r0:r1], vhead)
            nbytes = lib.nfi_render_backward_workspace_bytes(ctypes.byref(a))
            if nbytes < 0:
                _lib.check(-1, 'nfi_render_backward_workspace_bytes')
            ws = torch.empty((nbytes,), device=dev, dtype=torch.uint8)
            if DEBUG_BACKWARD is not None:      # diagnostics: the backward workspace (per-sample state)
                DEBUG_BACKWARD['workspace'] = ws
            tc = None if tile_counts is None else tile_counts[b0 * per_img:(b0 + nb) * per_img]
            g = _lib.NfiRenderGradArgs(
                g_rgb=_ptr(g_rgb[r0:r1]), g_mask=_ptr(g_mask[r0:r1]), d_planes=_ptr(d_planes[b0:b0 + nb]),
                d_palette_ray=_ptr(None if d_pal_ray is None else d_pal_ray[r0 * npl:r1 * npl]),
                g_ro=_ptr(None if g_ro is None else g_ro[r0:r1]), g_rd=_ptr(None if g_rd is None else g_rd[r0:r1]),
                tile_counts=_ptr(tc), workspace=_ptr(ws), workspace_bytes=nbytes,
                d_xray=_ptr(None if d_xray is None else d_xray[r0 * npl:r1 * npl]))
            return a, g, ws

        def stage(p, k, name, strm):
            a, g, _ = p
            with _timed(name, dev, strm):
                _lib.check(lib.nfi_render_backward_stage(ctypes.byref(a), ctypes.byref(g), k,
                                                         ctypes.c_void_p(strm.cuda_stream)),
                           'nfi_render_backward_stage')

        try:
            main = torch.cuda.current_stream(dev)
            if BACKWARD_PIPELINE and B >= 2 and DEBUG_BACKWARD is None:
                # two image halves: the tile pass of half 0 (VALU / LDS / gather bound) runs on a side
                # stream beside the field backward of half 1 (matrix-core bound)
                parts = [part(0, B // 2), part(B // 2, B - B // 2)]
                side = _side_stream(dev)
                events = []
                for p in parts:
                    stage(p, 0, 'bwd_bins', main)
                    stage(p, 1, 'bwd_field', main)
                    ev = torch.cuda.Event()
                    ev.record(main)
                    events.append(ev)
                for p, ev in zip(parts, events):
                    side.wait_event(ev)
                    stage(p, 2, 'bwd_tiles', side)
                    p[2].record_stream(side)
                for t in (d_planes, g_ro, g_rd, t_saved, tile_counts, planes_tm, ro, rd, near, far):
                    if t is not None:
                        t.record_stream(side)
                main.wait_stream(side)
            elif 0 < BACKWARD_SLAB < B and DEBUG_BACKWARD is None:
                for b0 in range(0, B, BACKWARD_SLAB):
                    p = part(b0, min(BACKWARD_SLAB, B - b0))
                    for k, name in enumerate(('bwd_bins', 'bwd_field', 'bwd_tiles')):
                        stage(p, k, name, main)
            else:
                p = part(0, B)
                for k, name in enumerate(('bwd_bins', 'bwd_field', 'bwd_tiles')):
                    stage(p, k, name, main)
        finally:
            lib.nfi_set_deterministic(prev_det)
        st = _stream(dev)
        d_pal = None
        if pal is not None:
            d_pal = torch.empty((B, 30), device=dev)
            ws = torch.empty((B * 64 * 30,), device=dev)
            _lib.check(lib.nfi_segment_sum(_ptr(d_pal_ray), B, H * W * npl, 30, _ptr(d_pal), _ptr(ws), st),
                       'nfi_segment_sum')
            d_pal = d_pal.view(B, 10, 3)
        d_ro = g_ro.view(B, H, W, 3) if need_coords else None
        d_rd = g_rd.view(B, H, W, 3) if need_coords else None
        d_xr = None
        if xray is not None and ctx.needs_input_grad[12]:
            d_xr = d_xray.view(n, npl, 32).sum(dim=1).view(xray.shape)
        return (d_planes, d_pal, d_ro, d_rd, None, None, None, None, None, None, None, None, d_xr, None)


def volume_render(planes_tm, palette, ro, rd, near, far, dec, opts: RenderOptions,
                  u_coarse=None, u_fine=None, seed: Optional[int] = None, debug: Optional[dict] = None,
                  xray=None, vhead=None):
    """Fused coarse+fine render of rays (run.py:202-348).  planes_tm: texel-major
    [B,3,R,R,32] (see planes_texel_major); palette [B,10,3] (None with opts.heads &
    HEAD_RGB_SIGMOID); ro, rd [B,H,W,3]; near, far
    [B,H,W].  Returns rgb [B,H,W,3], depth [B,H,W] (no grad), mask [B,H,W]; with opts.extras
    also the normal map [B,H,W,3] and the semantic [B,H,W,10] / coords [B,H,W,3] map (no grad;
    None when not requested).  opts.heads & HEAD_VIEWDIR: xray [B,H,W,32] is the per-ray
    view-direction mapper trunk output (differentiable) and vhead its packed output layer
    (pack_viewdir_head); dec is then a 33-output decoder."""
    _require_device(planes_tm, palette, ro, rd, near, far, dec, u_coarse, u_fine, xray, vhead)
    if bool(opts.heads & HEAD_VIEWDIR) != (xray is not None and vhead is not None):
        raise ValueError('xray and vhead are required exactly with HEAD_VIEWDIR')
    nout = 33 if opts.heads & HEAD_VIEWDIR else 11
    if dec.numel() != int(_lib.load().nfi_decoder_size(nout)):
        raise ValueError(f'packed decoder has {dec.numel()} floats; the field needs a {nout}-output decoder')
    if xray is not None:
        if xray.shape != (*ro.shape[:3], 32):
            raise ValueError(f'xray must be [B,H,W,32], got {tuple(xray.shape)}')
        if vhead.numel() != (3 if opts.heads & HEAD_RGB_SIGMOID else 10) * 33:
            raise ValueError('vhead must hold the [O,32] weights and [O] bias of the mapper output layer')
    if planes_tm.dim() != 5 or planes_tm.shape[-1] != 32 or planes_tm.stride(-1) != 1:
        raise ValueError('planes_tm must be texel-major [B,3,R,R,32] with unit channel stride')
    if planes_tm.stride(2) != planes_tm.shape[3] * planes_tm.stride(3):
        raise ValueError('planes_tm rows must be dense (stride(2) == R*stride(3))')
    if planes_tm.data_ptr() % 16 or any(st % 4 for st in planes_tm.stride()[:4]):
        raise ValueError('planes_tm must be 16-byte aligned with texel/plane/batch strides '
                         'divisible by 4 (the kernels load channel quads as float4)')
    B = planes_tm.shape[0]
    if (palette is None) != bool(opts.heads & HEAD_RGB_SIGMOID):
        raise ValueError('a palette is required exactly when the colour head is the attention head')
    if ro.shape[0] != B or (palette is not None and palette.shape != (B, 10, 3)):
        raise ValueError('batch mismatch between planes, palette and rays')
    n = ro.shape[0] * ro.shape[1] * ro.shape[2]
    if opts.randomize and (DEVICE_DRAWS or torch.cuda.is_current_stream_capturing()):
        # a captured HIP graph replays its launch arguments: a host-drawn Philox seed would repeat
        # on every replay, so the draws come from torch's graph-safe device generator instead
        # (fresh on each replay; the same U[0,1) the kernels' own Philox stream provides)
        if u_coarse is None:
            u_coarse = torch.rand(n * opts.samples, device=ro.device)
        if u_fine is None and opts.fine:
            u_fine = torch.rand(n * opts.samples, device=ro.device)
    for name, u in (('u_coarse', u_coarse), ('u_fine', u_fine)):
        if u is not None and u.numel() != n * opts.samples:
            raise ValueError(f'{name} must have B*H*W*S = {n * opts.samples} elements')
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if opts.randomize else 0
    rgb, depth, mask, nmap, smap = _VolumeRender.apply(planes_tm, palette, ro, rd, near, far, dec, opts,
                                                       u_coarse, u_fine, seed, debug, xray, vhead)
    if opts.extras:
        return rgb, depth, mask, (nmap if nmap.numel() else None), (smap if smap.numel() else None)
    return rgb, depth, mask
