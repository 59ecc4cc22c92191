"""Autograd operators over the producer C-ABI (include/nfi_producer.h): the fused HIP kernels
between the synthesis network's convolutions.  Device tensors only; the generator is frozen in
the inversion (run.py:630-632), so biases never receive gradients (asking for one raises).

  scale      x * s[b,c]                         stylegan.py:130 (modulation)
  act        lrelu(gain*(o*d[b,c] + bias[c]))   stylegan.py:145, 348-356 (demodulation epilogue)
  fir_up_act FIR(t) then act                    stylegan.py:99-103 + the epilogue (up layers)
  up_add     upsample2d(img) + c + bias[c]      stylegan.py:69-73, 380-381, 428-433 (skip image)
  up_conv    conv_transpose2d(x, w^T, stride 2)  stylegan.py:99-101: one GEMM over the 9 taps + scatter
  up_conv_act  fir_up_act(up_conv(x, w))         the up layer tail fused (2n >= 64), fused backward
  modulated_conv1x1  conv2d(x * s, w 1x1)        stylegan.py:363-384 (to-planes) as one batched GEMM
  vgg_epilogue relu(x + bias[c]) (+ 2x2 max pool) LPIPS VGG16 trunk (lpips 0.1 via metrics.py:107)
  lpips_head   the LPIPS distance of one layer    metrics.py:130-146
  aug_sample   the 'vgg' loss's 15 augmented copies (run.py:720-767), gathered adjoint
"""

from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib, conv
from .ops import _require_device, _stream


def _p(t):
    return None if t is None else t.data_ptr()


_fns = {}


def _call(name, *args):
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(_lib.load(), name)
    rc = fn(*args)
    if rc:
        _lib.check(rc, name)


def _frozen(bias):
    if torch.is_grad_enabled() and bias.requires_grad:
        raise NotImplementedError('producer biases are frozen in the inversion path '
                                  '(call requires_grad_(False) on the generator)')


class _Scale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        _require_device(x, s)
        x = x.contiguous()
        s = s.contiguous()
        ctx.save_for_backward(x, s)
        return x * s[:, :, None, None]

    @staticmethod
    def backward(ctx, g):
        x, s = ctx.saved_tensors
        g = g.contiguous()
        B, C, H, W = x.shape
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ds = torch.empty((B, C), device=x.device, dtype=x.dtype)
        _call('nfi_syn_scale_backward', _p(g), _p(x), _p(s), _p(gx), _p(ds), B * C, H * W,
              _stream(x.device))
        return gx, ds


class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, o, d, bias, gain: float):
        _require_device(o, d, bias)
        _frozen(bias)
        o = o.contiguous()
        d = d.contiguous()
        B, C, H, W = o.shape
        y = torch.empty_like(o)
        _call('nfi_syn_act_forward', _p(o), _p(d), _p(bias), _p(y), B * C, C, H * W,
              ctypes.c_float(gain), _stream(o.device))
        ctx.save_for_backward(o, d, bias)
        ctx.gain = gain
        return y

    @staticmethod
    def backward(ctx, g):
        o, d, bias = ctx.saved_tensors
        g = g.contiguous()
        B, C, H, W = o.shape
        go = torch.empty_like(o)
        dd = torch.empty_like(d)
        _call('nfi_syn_act_backward', _p(g), _p(o), _p(d), _p(bias), _p(go), _p(dd), B * C, C,
              H * W, ctypes.c_float(ctx.gain), _stream(o.device))
        return go, dd, None, None


class _FirUpAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, d, bias, gain: float):
        _require_device(t, d, bias)
        _frozen(bias)
        t = t.contiguous()
        d = d.contiguous()
        B, C, T, T2 = t.shape
        assert T == T2 and T % 2 == 1
        n = (T - 1) // 2
        o = torch.empty((B, C, 2 * n, 2 * n), device=t.device, dtype=t.dtype)
        y = torch.empty_like(o)
        _call('nfi_syn_fir_up_act_forward', _p(t), _p(d), _p(bias), _p(o), _p(y), B * C, C, n,
              ctypes.c_float(gain), _stream(t.device))
        ctx.save_for_backward(o, d, bias)
        ctx.gain = gain
        return y

    @staticmethod
    def backward(ctx, g):
        o, d, bias = ctx.saved_tensors
        g = g.contiguous()
        B, C, H, W = o.shape
        n = H // 2
        go = torch.empty_like(o)
        dd = torch.empty_like(d)
        dev = _stream(o.device)
        _call('nfi_syn_act_backward', _p(g), _p(o), _p(d), _p(bias), _p(go), _p(dd), B * C, C,
              H * W, ctypes.c_float(ctx.gain), dev)
        gt = torch.empty((B, C, 2 * n + 1, 2 * n + 1), device=o.device, dtype=o.dtype)
        _call('nfi_syn_fir_up_backward', _p(go), _p(gt), B * C, n, dev)
        return gt, dd, None, None


def _up_weights(w):
    """(W9 [9*Co, Ci] = w[co, ci, ky, kx] at row (3ky+kx)*Co + co, and W9^T contiguous) of a
    frozen w, cached on the tensor per storage version — each as (fp32 matrix, split-f16 halves for
    conv.split_matmul_shared or None)."""
    key = (w.data_ptr(), w._version, w.device, conv.SPLIT16)
    hit = getattr(w, '_nfi_upconv', None)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            co, ci = w.shape[:2]
            W9 = w.detach().permute(2, 3, 0, 1).reshape(9 * co, ci).contiguous()
            W9t = W9.t().contiguous()
            hit = (key, ((W9, conv.split_matrix(W9)), (W9t, conv.split_matrix(W9t))))
        w._nfi_upconv = hit
    return hit[1]


_SLOT_OWNERS = {}


def _slot_owner(Wm):
    """The per-stream maxima buffers of one cached split matrix (keyed by its hi-halves tensor)."""
    return _SLOT_OWNERS.setdefault(Wm[1][0].data_ptr(), {})


def _mm_shared(Wm, X):
    """Wm[0] X[b] per image: the split GEMM when Wm carries halves and the maps have >= 1024 pixels,
    else torch.matmul (hipBLASLt).  Below 1024 the products are launch-sized (20-60 us) and hipBLASLt's
    small tiles fill the GPU better: scripts/gemm_bench.py, N = 16..256 split 1.1-2.4x slower, N >= 1024
    1.3-1.9x faster."""
    if Wm[1] is not None and X.shape[2] >= 1024:
        return conv.split_matmul_shared(Wm[1], X)
    return torch.matmul(Wm[0], X)


class _UpConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W9, W9t):
        x = x.contiguous()
        B, Ci, n, _ = x.shape
        Co = W9[0].shape[0] // 9
        P = _mm_shared(W9, x.view(B, Ci, n * n))                            # [B, 9*Co, n*n]
        t = torch.empty((B, Co, 2 * n + 1, 2 * n + 1), device=x.device, dtype=x.dtype)
        _call('nfi_syn_up_conv_scatter', _p(P), _p(t), B, Co, n, _stream(x.device))
        ctx.W9t = W9t            # (frozen: no saved-tensor version check needed)
        ctx.shape = (B, Ci, Co, n)
        return t

    @staticmethod
    def backward(ctx, gt):
        W9t = ctx.W9t
        B, Ci, Co, n = ctx.shape
        gt = gt.contiguous()
        dP = torch.empty((B, 9 * Co, n * n), device=gt.device, dtype=gt.dtype)
        _call('nfi_syn_up_conv_gather', _p(gt), _p(dP), B, Co, n, _stream(gt.device))
        return _mm_shared(W9t, dP).view(B, Ci, n, n), None, None           # conv_transpose2d's adjoint


def up_conv(x, w):
    """F.conv_transpose2d(x, w.transpose(0, 1), stride=2) for w [Co, Ci, 3, 3] (stylegan.py:99-101,
    the synthesis up-sampling layers) as GEMMs over the 9 taps: forward P = W9 x (the split-f16 GEMM,
    conv.split_matmul_shared; hipBLASLt fp32 with NFI_SPLIT16=0 or channel counts off multiples of 32 —
    125-137 TFLOP/s on the 256^2 generator's layers where MIOpen's transposed kernels reach 50-70)
    and the tap scatter nfi_syn_up_conv_scatter; data gradient W9^T dP after the tap gather
    nfi_syn_up_conv_gather.  A weight that takes gradients goes to MIOpen's conv_transpose2d."""
    _require_device(x, w)
    if torch.is_grad_enabled() and w.requires_grad:
        return F.conv_transpose2d(x, w.transpose(0, 1), stride=2)
    W9, W9t = _up_weights(w)
    return _UpConv.apply(x, W9, W9t)


class _UpConvAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W9, W9t, d, bias, gain: float):
        _frozen(bias)
        x = x.contiguous()
        d = d.contiguous()
        B, Ci, n, _ = x.shape
        Co = W9[0].shape[0] // 9
        P = _mm_shared(W9, x.view(B, Ci, n * n))                            # [B, 9*Co, n*n]
        o = torch.empty((B, Co, 2 * n, 2 * n), device=x.device, dtype=x.dtype)
        y = torch.empty_like(o)
        _call('nfi_syn_up_conv_fir_act_forward', _p(P), _p(d), _p(bias), _p(o), _p(y), B, Co, n,
              ctypes.c_float(gain), _stream(x.device))
        ctx.save_for_backward(o, d, bias)
        ctx.W9t = W9t
        ctx.gain = gain
        ctx.shape = (B, Ci, Co, n)
        return y

    @staticmethod
    def backward(ctx, g):
        o, d, bias = ctx.saved_tensors
        W9t = ctx.W9t
        B, Ci, Co, n = ctx.shape
        g = g.contiguous()
        dev = _stream(o.device)
        dd = torch.empty_like(d)
        dP = torch.empty((B, 9 * Co, n * n), device=o.device, dtype=o.dtype)
        slots = None
        if n % 32 == 0 and W9t[1] is not None and n * n >= 1024:
            # the fused pass also leaves max|dP| for the split product W9^T dP (no maximum pass)
            slots = conv.stream_slots(_slot_owner(W9t), o.device)
            _call('nfi_syn_up_conv_act_backward_max', _p(g), _p(o), _p(d), _p(bias), _p(dP), _p(dd), _p(slots), B,
                  Co, n, ctypes.c_float(ctx.gain), dev)
        elif n % 32 == 0:     # epilogue backward + FIR adjoint + tap gather in one pass
            _call('nfi_syn_up_conv_act_backward', _p(g), _p(o), _p(d), _p(bias), _p(dP), _p(dd), B, Co, n,
                  ctypes.c_float(ctx.gain), dev)
        else:
            go = torch.empty_like(o)
            _call('nfi_syn_act_backward', _p(g), _p(o), _p(d), _p(bias), _p(go), _p(dd), B * Co, Co,
                  4 * n * n, ctypes.c_float(ctx.gain), dev)
            gt = torch.empty((B, Co, 2 * n + 1, 2 * n + 1), device=o.device, dtype=o.dtype)
            _call('nfi_syn_fir_up_backward', _p(go), _p(gt), B * Co, n, dev)
            _call('nfi_syn_up_conv_gather', _p(gt), _p(dP), B, Co, n, dev)
        if slots is not None:
            gx = conv.split_matmul_shared(W9t[1], dP, slots).view(B, Ci, n, n) if ctx.needs_input_grad[0] else None
            if gx is None:   # (the maxima were left for a product that did not run: clear them)
                slots.zero_()
        else:
            gx = _mm_shared(W9t, dP).view(B, Ci, n, n) if ctx.needs_input_grad[0] else None
        return gx, None, None, dd, None, None


def up_conv_act(x, w, d, bias, gain: float):
    """The up-sampling layer after the modulation: fir_up_act(up_conv(x, w), d, bias, gain)
    (stylegan.py:99-103 + the demodulation epilogue :145, :348-356).  For 2n >= 64 the tap scatter,
    FIR and epilogue are one kernel (nfi_syn_up_conv_fir_act_forward: the (2n+1)^2 transposed-conv
    output never reaches HBM); smaller layers run the separate kernels."""
    _require_device(x, w, d, bias)
    n = x.shape[-1]
    if (2 * n) % 64 or (torch.is_grad_enabled() and w.requires_grad):
        return fir_up_act(up_conv(x, w), d, bias, gain)
    W9, W9t = _up_weights(w)
    return _UpConvAct.apply(x, W9, W9t, d, bias, gain)


# the planes layer's backward as one K = 96 product (round 5) instead of one product per plane plus
# in-place accumulations; NFI_PLANES_BWD_ONE=0 restores the per-plane form (A/B)
PLANES_BWD_ONE = os.environ.get('NFI_PLANES_BWD_ONE', '1') != '0'
# the augmentation grid in one launch (nfi_aug_affine_grid); NFI_AFFINE_GRID_HIP=0: F.affine_grid
AFFINE_GRID_HIP = os.environ.get('NFI_AFFINE_GRID_HIP', '1') != '0'


class _ModConv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s, Wf, Wt, layout: str):
        x = x.contiguous()
        s = s.contiguous()
        B, C, H, W = x.shape
        O = Wf.shape[0]
        Wm = Wf[None] * s[:, None, :]                                       # [B, O, C]
        if layout != 'nchw':  # y^T = x^T Wm^T: [B, HW, O], i.e. [B, O, H, W] in channels-last strides
            y = torch.bmm(x.view(B, C, H * W).transpose(1, 2), Wm.transpose(1, 2))
            y = (y.view(B, H, W, O).permute(0, 3, 1, 2) if layout == 'nhwc'
                 else y.view(B, H, W, O // 32, 32).permute(0, 3, 4, 1, 2))      # 'planes': [B, O/32, 32, H, W]
        else:
            y = torch.bmm(Wm, x.view(B, C, H * W)).view(B, O, H, W)
        ctx.save_for_backward(x, s, Wt)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, s, Wt = ctx.saved_tensors
        B, C, H, W = x.shape
        if gy.dim() == 5 and not PLANES_BWD_ONE:   # (the round-4 form: one product per plane, accumulated)
            gxs = None
            for q in range(gy.shape[1]):
                gq = gy[:, q].reshape(B, 32, H * W)
                Wq = Wt[:, 32 * q:32 * (q + 1)]
                gxs = torch.matmul(Wq, gq) if gxs is None else gxs.baddbmm_(Wq.expand(B, -1, -1), gq)
        elif gy.dim() == 5:   # texel-major planes [B, Q, 32, H, W]: the Q planes' channels are one
            # K = 32 Q contraction — one product instead of a product + Q - 1 in-place accumulations over
            # the [B, C, HW] result.  The texel-major gradient ([B][Q][HW][32] in memory) is not a K x HW
            # matrix (plane stride HW*32, channel stride 1): it goes channel-major by the renderer's
            # LDS-tiled conversion (nfi_planes_to_channel_major) — a reshape here made ATen's strided
            # copy, 113 us per step for the 100 MB at B = 4
            Q = gy.shape[1]
            if Q == 3 and H == W and gy.permute(0, 1, 3, 4, 2).is_contiguous():
                gc = torch.empty((B, 3 * 32, H * W), device=gy.device, dtype=gy.dtype)
                _call('nfi_planes_to_channel_major', _p(gy), B, H, _p(gc), _stream(gy.device))
            else:
                gc = gy.reshape(B, Q * gy.shape[2], H * W)
            gxs = torch.matmul(Wt, gc)
        elif gy.is_contiguous():
            gxs = torch.matmul(Wt, gy.view(B, -1, H * W))
        else:                 # channels-last: [B, HW, O] seen as [B, O, HW] (a transposed operand, no copy)
            gxs = torch.matmul(Wt, gy.permute(0, 2, 3, 1).reshape(B, H * W, -1).transpose(1, 2))
        # gxs = d(x * s) [B, C, HW]
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ds = torch.empty((B, C), device=x.device, dtype=x.dtype)
        _call('nfi_syn_scale_backward', _p(gxs), _p(x), _p(s), _p(gx), _p(ds), B * C, H * W,
              _stream(x.device))
        return gx, ds, None, None, None


def modulated_conv1x1(x, s, weight, layout: str = 'nchw'):
    """F.conv2d(x * s[:, :, None, None], weight) for a frozen 1x1 weight [O, C, 1, 1] (the toRGB /
    to-planes layers, stylegan.py:363-384): the modulation goes into a per-image weight (W * s_b,
    [B, O, C]: O = 96 rows, far smaller than x) and the layer is one batched GEMM; the backward is
    W^T dy (one GEMM) and nfi_syn_scale_backward (d x = s * that, d s = sum x * that).
    layout 'nhwc' returns [B, O, H, W] in channels-last strides (the skip-image chain's layout);
    'planes' returns it as [B, O/32, 32, H, W] (the last layer's: up_add then writes the renderer's
    texel-major planes).  A weight that takes gradients goes to MIOpen."""
    _require_device(x, s, weight)
    if torch.is_grad_enabled() and weight.requires_grad:
        return F.conv2d(x * s[:, :, None, None], weight)
    key = (weight.data_ptr(), weight._version, weight.device)
    hit = getattr(weight, '_nfi_1x1', None)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            Wf = weight.detach().reshape(weight.shape[0], -1).contiguous()
            hit = (key, (Wf, Wf.t().contiguous()))
        weight._nfi_1x1 = hit
    if layout not in ('nchw', 'nhwc', 'planes') or (layout == 'planes' and weight.shape[0] % 32):
        raise ValueError(f'modulated_conv1x1: layout {layout!r} for {weight.shape[0]} outputs')
    return _ModConv1x1.apply(x, s, *hit[1], layout)


class _AugSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, grid, copies: int, shift: float):
        img = img.contiguous()
        grid = grid.contiguous()
        B, H, W, _ = img.shape
        Ho, Wo = grid.shape[1:3]
        out = torch.empty((B * copies, 3, Ho, Wo), device=img.device, dtype=img.dtype)
        _call('nfi_aug_sample_forward', _p(img), _p(grid), _p(out), B, copies, H, W, Ho, Wo,
              ctypes.c_float(shift), _stream(img.device))
        ctx.save_for_backward(grid)
        ctx.shape = (B, copies, H, W, Ho, Wo)
        return out

    @staticmethod
    def backward(ctx, gout):
        grid, = ctx.saved_tensors
        B, K, H, W, Ho, Wo = ctx.shape
        gout = gout.contiguous()
        gimg = torch.empty((B, H, W, 3), device=gout.device, dtype=gout.dtype)
        _call('nfi_aug_sample_backward', _p(gout), _p(grid), _p(gimg), B, K, H, W, Ho, Wo, _stream(gout.device))
        return gimg, None, None, None


def affine_grid(theta, size):
    """F.affine_grid(theta, size, align_corners=False) for theta [N, 2, 3] on the device, size
    [N, C, H, W] (augment_impl's grid, run.py:749): one launch (nfi_aug_affine_grid) instead of ATen's
    base grid + batched product.  No gradient (the augmentation parameters are random draws)."""
    _require_device(theta)
    N, _, H, W = size
    if theta.shape != (N, 2, 3) or theta.dtype != torch.float32:
        raise ValueError(f'affine_grid: theta {tuple(theta.shape)} {theta.dtype} for size {tuple(size)}')
    theta = theta.detach().contiguous()
    grid = torch.empty((N, H, W, 2), device=theta.device, dtype=theta.dtype)
    _call('nfi_aug_affine_grid', _p(theta), N, H, W, _p(grid), _stream(theta.device))
    return grid


def aug_sample(img, grid, copies: int, white_background: bool = False):
    """The 'vgg' loss's augmented copies (run.py:720-767, 2211-2235): img [B, H, W, 3] (channels
    last, as rendered) -> [B*copies, 3, Ho, Wo] = grid_sample(img[b] (- 1), grid[b*copies + k],
    bilinear, zeros, align_corners=False) (+ 1 on white backgrounds), without materializing the
    expanded copies; the backward gathers each input pixel's share from all copies (no atomics,
    nfi_aug_sample_backward) into d img [B, H, W, 3].  Each copy's grid must be affine in the
    output pixel (F.affine_grid, as inversion.augment_grid builds it): the adjoint enumerates the
    preimage of each input pixel's neighbourhood under that map."""
    _require_device(img, grid)
    if img.shape[-1] != 3 or grid.shape[0] != img.shape[0] * copies or grid.shape[-1] != 2:
        raise ValueError(f'aug_sample: img {tuple(img.shape)} / grid {tuple(grid.shape)} / copies {copies}')
    return _AugSample.apply(img, grid.detach(), copies, 1.0 if white_background else 0.0)


def _str3(t):
    """(b, q, t) float strides of a channel-contiguous [B, C, h, w] (channels-last) or
    [B, C/32, 32, h, w] (texel-major planes) tensor, as the strided C-ABI takes them; None if t is
    neither."""
    if t.dim() == 4 and t.stride(1) == 1 and t.stride(2) == t.shape[3] * t.stride(3):
        return (ctypes.c_int64 * 3)(t.stride(0), 32, t.stride(3))
    if t.dim() == 5 and t.shape[2] == 32 and t.stride(2) == 1 and t.stride(3) == t.shape[4] * t.stride(4):
        return (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(4))
    return None


def _conform(t):
    """t in a layout _str3 accepts (a copy only if it is in neither)."""
    if _str3(t) is not None:
        return t
    if t.dim() == 4:
        return t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)


def _texel_major(shape, dev, dtype):
    """[B, Q, 32, h, w] stored as [B, Q, h, w, 32] (the renderer's plane layout)."""
    B, Q, _, h, w = shape
    return torch.empty((B, Q, h, w, 32), device=dev, dtype=dtype).permute(0, 1, 4, 2, 3)


class _UpAddStrided(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, c, bias):
        _require_device(img, c, bias)
        _frozen(bias)
        c = _conform(c)
        B = c.shape[0]
        C = c.shape[1] * (c.shape[2] if c.dim() == 5 else 1)
        H = c.shape[-2]
        n = H // 2
        if img is not None:
            img = img.contiguous(memory_format=torch.channels_last)
            assert img.shape == (B, C, n, n), (img.shape, c.shape)
        # a 5-d c (the last layer's to-planes output) -> texel-major planes; else channels-last
        out = (_texel_major(c.shape, c.device, c.dtype) if c.dim() == 5
               else torch.empty_like(c, memory_format=torch.channels_last))
        _call('nfi_syn_up_add_forward_strided', _p(img), None if img is None else _str3(img), _p(c), _str3(c),
              _p(bias.contiguous()), _p(out), _str3(out), B, C, n, _stream(c.device))
        ctx.has_img = img is not None
        ctx.shape = (B, C, n)
        return out

    @staticmethod
    def backward(ctx, g):
        gimg = None
        g = _conform(g)
        if ctx.has_img and ctx.needs_input_grad[0]:
            B, C, n = ctx.shape
            gimg = torch.empty((B, C, n, n), device=g.device, dtype=g.dtype, memory_format=torch.channels_last)
            _call('nfi_syn_up_backward_strided', _p(g), _str3(g), _p(gimg), _str3(gimg), B, C, n, _stream(g.device))
        return gimg, g, None


class _UpAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, c, bias):
        _require_device(img, c, bias)
        _frozen(bias)
        c = c.contiguous()
        B, C, H, W = c.shape
        n = H // 2
        if img is not None:
            img = img.contiguous()
            assert img.shape == (B, C, n, n), (img.shape, c.shape)
        out = torch.empty_like(c)
        _call('nfi_syn_up_add_forward', _p(img), _p(c), _p(bias), _p(out), B * C, C, n,
              _stream(c.device))
        ctx.has_img = img is not None
        ctx.shape = (B, C, n)
        return out

    @staticmethod
    def backward(ctx, g):
        gimg = None
        if ctx.has_img and ctx.needs_input_grad[0]:
            g = g.contiguous()
            B, C, n = ctx.shape
            gimg = torch.empty((B, C, n, n), device=g.device, dtype=g.dtype)
            _call('nfi_syn_up_backward', _p(g), _p(gimg), B * C, n, _stream(g.device))
        return gimg, g, None


class _LpipsHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f0, f1, w):
        _require_device(f0, f1, w)
        f0 = f0.contiguous()
        f1 = f1.detach().contiguous()
        w = w.detach().contiguous()
        N, C, H, W = f0.shape
        out = torch.empty(N, device=f0.device, dtype=f0.dtype)
        inv0 = torch.empty(N * H * W, device=f0.device, dtype=f0.dtype)
        inv1 = torch.empty_like(inv0)
        _call('nfi_lpips_head_forward', _p(f0), _p(f1), _p(w), _p(out), _p(inv0), _p(inv1), N, C,
              H * W, _stream(f0.device))
        ctx.save_for_backward(f0, f1, w, inv0, inv1)
        return out

    @staticmethod
    def backward(ctx, g):
        f0, f1, w, inv0, inv1 = ctx.saved_tensors
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            raise NotImplementedError('lpips_head differentiates the first input only')
        g = g.contiguous()
        N, C, H, W = f0.shape
        gf0 = torch.empty_like(f0)
        _call('nfi_lpips_head_backward', _p(g), _p(f0), _p(f1), _p(w), _p(inv0), _p(inv1), _p(gf0),
              N, C, H * W, _stream(f0.device))
        return gf0, None, None


class _VggEpilogue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, pool: bool):
        _require_device(x, bias)
        _frozen(bias)
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty_like(x)
        m = torch.empty((N, C, H // 2, W // 2), device=x.device, dtype=x.dtype) if pool else None
        _call('nfi_vgg_bias_relu_forward', _p(x), _p(bias.detach().contiguous()), _p(y), _p(m),
              N * C, C, H, W, _stream(x.device))
        ctx.save_for_backward(y)
        ctx.set_materialize_grads(False)       # an unused output's gradient arrives as None
        return (y, m) if pool else y

    @staticmethod
    def backward(ctx, gy, gm=None):
        y, = ctx.saved_tensors
        if gy is None and gm is None:
            return None, None, None
        N, C, H, W = y.shape
        gx = torch.empty_like(y)
        gy = None if gy is None else gy.contiguous()
        gm = None if gm is None else gm.contiguous()
        _call('nfi_vgg_relu_backward', _p(gy), _p(gm), _p(y), _p(gx), N * C, H, W, _stream(y.device))
        return gx, None, None


class _VggFirst(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, shift=None, scale=None):
        x = x.contiguous()
        N, _, H, W = x.shape
        Co = w.shape[0]
        y = torch.empty((N, Co, H, W), device=x.device, dtype=x.dtype)
        wd = w.detach().contiguous()
        sh = None if shift is None else shift.detach().reshape(3).contiguous()
        sc = None if scale is None else scale.detach().reshape(3).contiguous()
        # each image's max of y for the next layer's direct convolution (nfi.conv._direct)
        from .conv import slot_words
        ymax = torch.zeros((slot_words(),), device=x.device, dtype=torch.int32)
        _call('nfi_vgg_first_forward_max', _p(x), _p(sh), _p(sc), _p(wd), _p(bias.detach().contiguous()), _p(y),
              _p(ymax), N, Co, H, W, _stream(x.device))
        y._nfi_absmax = (ymax, y._version, y.data_ptr())
        ctx.save_for_backward(y, wd, sc)
        return y

    @staticmethod
    def backward(ctx, gy):
        y, wd, sc = ctx.saved_tensors
        N, Co, H, W = y.shape
        gx = torch.empty((N, 3, H, W), device=y.device, dtype=y.dtype)
        _call('nfi_vgg_first_backward_scaled', _p(gy.contiguous()), _p(y), _p(wd), _p(sc), _p(gx), N, Co, H, W,
              _stream(y.device))
        return gx, None, None, None, None


def vgg_first_applicable(x, w) -> bool:
    return (x.dim() == 4 and x.shape[1] == 3 and tuple(w.shape[1:]) == (3, 3, 3) and x.shape[-2] % 16 == 0
            and x.shape[-1] % 64 == 0 and not (torch.is_grad_enabled() and w.requires_grad))


def vgg_first(x, w, bias, shift=None, scale=None):
    """relu(conv2d(x', w, bias, padding=1)) for the LPIPS trunk's 3-channel first layer
    (vgg16.features[0:2]), x' = x or, with shift / scale ([3] or [1, 3, 1, 1]), the ScalingLayer's
    (x - shift) / scale (lpips 0.1) folded into the same pass: one direct-convolution pass with the
    epilogue each way (nfi_vgg_first_forward_max / _backward_scaled); frozen weights (the LPIPS net is
    not trained)."""
    _require_device(x, w, bias)
    _frozen(bias)
    return _VggFirst.apply(x, w, bias, shift, scale)


def vgg_epilogue(x, bias, pool: bool = False):
    """relu(x + bias[c]) of a bias-free conv output x; with pool=True also returns MaxPool2d(2, 2)
    of it: (y, pooled).  One HIP pass each way (nfi_vgg_bias_relu_forward / nfi_vgg_relu_backward)."""
    return _VggEpilogue.apply(x, bias, pool)


class _CondNormAct(torch.autograd.Function):
    """lrelu(beta + gamma1 * layer_norm(h), 0.2) (generator.py:42-60, 173-178): one HIP kernel each
    way (nfi_syn_cond_norm_act_*) instead of layer_norm / addcmul / leaky_relu and their backwards.
    gamma1 and beta may be row-strided views of one [B, k*C] projection (their last dim contiguous)."""

    @staticmethod
    def forward(ctx, h, gamma1, beta):
        _require_device(h, gamma1, beta)
        h = h.contiguous()
        B, C = h.shape
        if gamma1.stride(-1) != 1 or beta.stride(-1) != 1 or gamma1.stride(0) != beta.stride(0):
            gamma1, beta = gamma1.contiguous(), beta.contiguous()
        ld = gamma1.stride(0)
        x = torch.empty_like(h)
        stats = torch.empty((B, 2), device=h.device)
        _call('nfi_syn_cond_norm_act_forward', _p(h), _p(gamma1), _p(beta), B, C, ld, _p(x), _p(stats),
              _stream(h.device))
        ctx.save_for_backward(h, gamma1, beta, stats)
        ctx.ld = ld
        return x

    @staticmethod
    def backward(ctx, gx):
        h, gamma1, beta, stats = ctx.saved_tensors
        B, C = h.shape
        dh, dg1, db = torch.empty_like(h), torch.empty_like(h), torch.empty_like(h)
        _call('nfi_syn_cond_norm_act_backward', _p(gx.contiguous()), _p(h), _p(gamma1), _p(beta), _p(stats), B, C,
              ctx.ld, _p(dh), _p(dg1), _p(db), _stream(h.device))
        return dh, dg1, db


def cond_norm_act(h, gamma1, beta):
    """F.leaky_relu(torch.addcmul(beta, gamma1, F.layer_norm(h, (C,))), 0.2) for [B, C] rows."""
    return _CondNormAct.apply(h, gamma1, beta)


def lpips_head(f0, f1, w):
    """[N] = mean_hw sum_c w_c (n(f0) - n(f1))_c^2 (lpips distance of one layer)."""
    return _LpipsHead.apply(f0, f1, w)


def scale(x, s):
    return _Scale.apply(x, s)


def act(o, d, bias, gain: float):
    return _Act.apply(o, d, bias, gain)


def fir_up_act(t, d, bias, gain: float):
    return _FirUpAct.apply(t, d, bias, gain)


def up_add(img, c, bias):
    """upsample2d(img) + c + bias (stylegan.py:69-73, 380-381, 428-433): NCHW; channels-last when c
    is; texel-major planes [B, C/32, 32, 2n, 2n] (the renderer's layout) when c is 5-d
    (nfi_syn_up_add_forward_strided)."""
    if c.dim() == 5 or (c.is_contiguous(memory_format=torch.channels_last) and not c.is_contiguous()
                        and c.shape[1] % 4 == 0):
        return _UpAddStrided.apply(img, c, bias)
    return _UpAdd.apply(img, c, bias)
