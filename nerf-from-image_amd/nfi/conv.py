"""3x3 convolutions of the inversion step's caller side as Winograd F(4x4, 3x3) on MI355X: the
LPIPS VGG16 trunk (lpips 0.1 via lib/metrics.py:107) and the synthesis layers
(models/stylegan.py:130-145, §8(f) #1) call F.conv2d(x, w, padding=1) with frozen weights
(run.py:630-632; LPIPS is never trained), in fp32 (TF32 off, run.py:59-60).

Per layer: input transform (HIP) -> 36 batched [Co x Ci] x [Ci x P] fp32-accurate GEMMs on the f16
matrix cores (nfi's split-f16 product, csrc/nfi_gemm.hip; torch.bmm / hipBLASLt with NFI_SPLIT16=0)
-> output transform (HIP, with the VGG block's bias + ReLU + 2x2 max pool fused); the 64-channel
layers as one fused HIP kernel.  The large maps (the LPIPS 128^2 and 64^2 layers, forward and data
gradient) run instead as a direct convolution on the f16 matrix cores (csrc/nfi_dconv.hip, same
split-f16 products, no Winograd round trips).  Weight transforms are computed once per frozen weight.  The
data gradient is the same pipeline with the rot180 / channel-swapped weights (the weights
receive no gradient: asking for one raises).  csrc/nfi_conv.hip, include/nfi_producer.h.

F(4,3) multiplies 4x fewer products than the direct convolution (MIOpen's fp32 Winograd is
F(2,3), 2.25x, on the vector ALUs).  Its transforms cost fp32 rounding: a few 1e-6 of the
largest output (tests/test_gpu_conv.py bounds it by 2e-5 against an fp64 convolution, next to
MIOpen's own error), the order of cuDNN's fp32 Winograd algorithms the reference may run.
"""

from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib
from .ops import _require_device, _stream

# layers with fewer input channels than this stay on MIOpen (the VGG trunk's 3-channel first
# layer: K = 3 is no GEMM)
MIN_CHANNELS = 16
ENABLED = True
DGRAD = True          # data gradient as Winograd too (False: MIOpen's conv2d_input; diagnostics)
FOLD_SCALE = os.environ.get('NFI_FOLD_SCALE', '1') == '1'   # modulation folded into the input transform
FUSED = True          # one fused kernel per layer (nfi_wino_conv_fused) for layers with Ci % 8 == 0
                      # and Ci <= FUSED_MAX_CI; else the three-pass form (transforms + hipBLASLt GEMM)
# The fused kernel keeps V and M on chip but its 36-way split accumulators leave small per-product
# tiles: 46-64 TFLOP/s of Winograd products on MI355X vs 100-137 for hipBLASLt's batched GEMM.  It
# wins where the three-pass form's HBM round trips dominate — the 64-channel, large-map layers
# (LPIPS 64->64 @128^2: 0.42 vs 0.68 ms; Ci = 128 is a per-layer tie that loses over the step:
# NFI_FUSED_MAX_CI=128 measured 18.9 vs 18.8 ms) — and loses on the deeper ones (512->512 @16^2: 0.32 vs
# 0.21 ms); scripts/wino_layers.py.
FUSED_MAX_CI = int(os.environ.get('NFI_FUSED_MAX_CI', '64'))
# ... and output channels: with the split-f16 GEMM (round 4) the three-pass form wins 64->128 @64^2
# (0.220 vs 0.263 ms) while the fused kernel keeps 64->64 @128^2 (0.48-0.51 vs 0.62 ms)
FUSED_MAX_CO = int(os.environ.get('NFI_FUSED_MAX_CO', '64'))


def _fused_ok(Uw, Ci, Co):
    """Whether a layer with these channel counts runs as the fused kernel."""
    return FUSED and Uw.packed is not None and Ci <= FUSED_MAX_CI and (Co <= FUSED_MAX_CO or not SPLIT16)
# the VGG blocks' ReLU threshold_backward inside the data gradient's input transform (no pool
# gradient; three-pass layers)
RELU_IN_TRANSFORM = os.environ.get('NFI_RELU_IN_TRANSFORM', '1') != '0'
# the three-pass layers' 36 products on the f16 matrix cores at fp32 accuracy (csrc/nfi_gemm.hip:
# hi / lo splits, three products each; the weights split once, V's scale from the input
# transform's running maximum); 0: torch.bmm (hipBLASLt fp32)
# B's power-of-two scale is PER IMAGE (round 6; csrc/nfi_gemm.hip): the input transform leaves each
# image's maximum |V| in that image's slots and the GEMM splits and unscales every column with its own
# image's scale, so an image's operand precision — and its result — does not depend on the other
# images of the batch, and a sharded run matches the unsharded one per image
# (tests/test_gpu_gemm.py::test_split16_per_image_scale).
SPLIT16 = os.environ.get('NFI_SPLIT16', '1') != '0'
SPLIT16_BK = 32       # the split GEMM's K step: channel counts must be multiples of it
KSPLIT = os.environ.get('NFI_KSPLIT', '1') != '0'   # K split of the Winograd products with few tiles
# the fused layers on the f16 matrix cores (nfi_wino_conv_fused_split: products consumed by the output
# transform one Winograd row at a time) where the shapes allow — measured slower than fused_kernel's
# fp32 MFMAs (0.68 vs 0.48-0.51 ms on the 64->64 @128^2 layer), so off unless NFI_FUSED_SPLIT=1
FUSED_SPLIT = os.environ.get('NFI_FUSED_SPLIT', '0') != '0'
# Direct convolution on the f16 matrix cores (csrc/nfi_dconv.hip, nfi_dconv3x3) for the large maps: the
# products as the split GEMM's, x's scale per image, no Winograd round trips through HBM.  Taken for
# layers with Ci % 16 == 0, Co % 64 == 0, H % 8 == 0, W % 64 == 0 and H*W >= DIRECT_MIN_HW (the LPIPS
# 128^2 and 64^2 maps) and no modulation scale (NFI_DCONV=0: the Winograd forms everywhere).
DIRECT = os.environ.get('NFI_DCONV', '1') != '0'
DIRECT_MIN_HW = int(os.environ.get('NFI_DCONV_MIN_HW', str(64 * 64)))
# ... and the modulated synthesis layers (the scale folded into the staging, csrc/nfi_dconv.hip xscale):
# measured SLOWER on the inversion step's 4-image producer (l1 8.32-8.35 vs 8.04-8.12 ms: the Winograd
# products of 4 images of 128 channels cost no more than the direct form's maxima pass + scale backward
# pass), so off unless NFI_DCONV_MOD=1 (tests/test_gpu_dconv.py covers it)
DIRECT_MOD = os.environ.get('NFI_DCONV_MOD', '0') != '0'


class WeightSet:
    """One orientation of a frozen 3x3 weight, transformed: U [36, M, K] fp32 (the hipBLASLt
    product), `packed` (the fused kernel's MFMA operands, or None), `split` = (hi, lo, inverse
    scales) f16 halves for the split-f16 product (or None) and `direct` = (packed halves, inverse
    scale) for the direct convolution nfi_dconv3x3 (or None)."""
    __slots__ = ('U', 'packed', 'split', 'direct', 'direct_src', 'vmax')

    def __init__(self, U, packed, split, direct=None, direct_src=None):
        self.U, self.packed, self.split, self.direct = U, packed, split, direct
        self.direct_src = direct_src   # (w, Co, Ci, flip): `direct` packed on first use (_direct_ok)
        self.vmax = {}   # stream -> the split product's maxima slots (self-clearing: see _slots)


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


def applicable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """True when conv2d(x, weight, padding=1) runs as Winograd here: a device tensor, 3x3 kernel,
    H and W multiples of 4, enough input channels for a GEMM."""
    return (ENABLED and x.is_cuda and x.dim() == 4 and weight.shape[2:] == (3, 3)
            and x.shape[1] >= MIN_CHANNELS and x.shape[2] % 4 == 0 and x.shape[3] % 4 == 0
            and x.dtype == torch.float32)


def weights(weight: torch.Tensor):
    """(U, Ut) of a frozen [Co,Ci,3,3] weight, cached until the weight is modified in place or
    replaced: each a (transformed [36,Co,Ci] or [36,Ci,Co], MFMA-packed or None) pair — the
    packed form (nfi_wino_pack_weights) feeds the fused kernel when its input-channel count is a
    multiple of 8."""
    tag = (weight.data_ptr(), weight._version, weight.device)
    hit = getattr(weight, '_nfi_winograd', None)
    if hit is not None and hit[0] == tag:
        return hit[1]
    _require_device(weight)
    w = weight.detach().contiguous()
    Co, Ci = w.shape[:2]
    U = torch.empty((36, Co, Ci), device=w.device)
    Ut = torch.empty((36, Ci, Co), device=w.device)
    st = _stream(w.device)
    _call('nfi_wino_weight_transform', _p(w), _p(U), Co, Ci, 0, st)
    _call('nfi_wino_weight_transform', _p(w), _p(Ut), Co, Ci, 1, st)
    out = (WeightSet(U, _pack(U, Co, Ci, st), _split(U, Ci, st), direct_src=(w, Co, Ci, False)),
           WeightSet(Ut, _pack(Ut, Ci, Co, st), _split(Ut, Co, st), direct_src=(w, Co, Ci, True)))
    weight._nfi_winograd = (tag, out)          # cached on the (frozen) parameter itself
    return out


def _split(U, K, st):
    """U [36, M, K] -> (hi, lo [36, M, K] f16 bits, inverse scales [36]) for nfi_gemm_split16."""
    if K % SPLIT16_BK:
        return None
    hi = torch.empty(U.shape, device=U.device, dtype=torch.int16)
    lo = torch.empty(U.shape, device=U.device, dtype=torch.int16)
    inv = torch.empty((U.shape[0],), device=U.device)
    _call('nfi_split16_pack', _p(U), U.shape[0], U.shape[1] * U.shape[2], _p(hi), _p(lo), _p(inv), st)
    return hi, lo, inv


def _direct_pack(w, Co, Ci, flip, st):
    """w [Co, Ci, 3, 3] -> (wp [2 * 9 * Ci * Co] f16 bits, w_inv [1]) for nfi_dconv3x3: the forward weight,
    or (flip) the data gradient's; None when its input channels are not a multiple of 16."""
    if not DIRECT or (Co if flip else Ci) % 16:
        return None
    wp = torch.empty((2 * 9 * Co * Ci,), device=w.device, dtype=torch.int16)
    winv = torch.empty((1,), device=w.device)
    _call('nfi_dconv_pack', _p(w), Co, Ci, 1 if flip else 0, _p(wp), _p(winv), st)
    return wp, winv


def _direct_ok(Uw, x):
    """Whether conv3x3(x) with this weight orientation runs as nfi_dconv3x3."""
    N, Ci, H, W = x.shape
    Co = Uw.U.shape[1]
    if not (DIRECT and Ci % 16 == 0 and Co % 64 == 0 and H % 8 == 0 and W % 64 == 0 and H * W >= DIRECT_MIN_HW):
        return False
    if Uw.direct is None and Uw.direct_src is not None:   # packed on the layer's first direct call
        w, co, ci, flip = Uw.direct_src
        Uw.direct = _direct_pack(w, co, ci, flip, _stream(w.device))
        Uw.direct_src = None
    return Uw.direct is not None


def _maxima_of(t):
    """The per-image max |t| slots a dconv epilogue left on t (tagged with t's version and storage), or
    None."""
    tag = getattr(t, '_nfi_absmax', None)
    if tag is not None and tag[1] == t._version and tag[2] == t.data_ptr():
        return tag[0]
    return None


def _direct(x, Uw, bias=None, pool=False, relu_y=None, scale=None):
    """conv3x3(x') on the direct kernel, x' = x or x where relu_y > 0; with bias the VGG epilogue
    (and the pooled map when pool): y or (y, pooled).  x's per-image maxima come from the dconv that
    produced it when it left them (the VGG blocks' chain), else from one maxima pass; the VGG epilogue
    leaves y's (a bound for pooled too) on both outputs for the next layer.  scale [N, Ci]: the
    convolution of x * scale[n, c] (the modulated synthesis layers), folded into the staging."""
    N, Ci, H, W = x.shape
    Co = Uw.U.shape[1]
    st = _stream(x.device)
    slots = _maxima_of(x) if scale is None else None
    if scale is not None:
        slots = torch.empty((slot_words(),), device=x.device, dtype=torch.int32)
        _call('nfi_absmax_scaled_slots', _p(x), _p(scale), N, Ci, H * W, _p(slots), st)
    elif slots is None:
        slots = torch.empty((slot_words(),), device=x.device, dtype=torch.int32)
        _call('nfi_absmax_slots', _p(x), N, Ci * H * W, _p(slots), st)
    y = torch.empty((N, Co, H, W), device=x.device)
    m = torch.empty((N, Co, H // 2, W // 2), device=x.device) if pool else None
    ymax = torch.zeros((slot_words(),), device=x.device, dtype=torch.int32) if bias is not None else None
    wp, winv = Uw.direct
    _call('nfi_dconv3x3', _p(x), _p(scale), _p(relu_y), _p(slots), _p(wp), _p(winv), _p(bias), _p(y), _p(m), _p(ymax), N, Ci, Co,
          H, W, st)
    if ymax is not None:
        for t in (y, m):
            if t is not None:
                t._nfi_absmax = (ymax, t._version, t.data_ptr())
    return (y, m) if pool else y


def _conv(x, Uw, bias=None, pool=False, scale=None):
    """The layer's convolution on its fastest form: the direct kernel where _direct_ok, else
    Winograd (fused or three-pass)."""
    if (scale is None or (DIRECT_MOD and bias is None and not pool)) and _direct_ok(Uw, x):
        return _direct(x, Uw, bias, pool, scale=scale)
    return _winograd(x, Uw, bias, pool, scale)


def split_matrix(A):
    """A frozen [M, K] fp32 matrix -> its split-f16 halves for split_matmul_shared (None when K is not
    a multiple of SPLIT16_BK, or SPLIT16 is off: the caller keeps torch.matmul)."""
    if not SPLIT16 or A.shape[1] % SPLIT16_BK:
        return None
    return _split(A.detach().contiguous()[None], A.shape[1], _stream(A.device))


_slot_words = None


def slot_words() -> int:
    """uint32 words of a split product's maxima buffer (nfi_split16_slot_words: 256 images x 4 slots
    + the completion counter)."""
    global _slot_words
    if _slot_words is None:
        _slot_words = int(_lib.load().nfi_split16_slot_words())
    return _slot_words


def split_matmul_shared(As, X, slots=None):
    """C[b] = A X[b] for X [B, K, N] on the split GEMM, A's halves from split_matrix (one A for every
    image: nfi_gemm_split16_shared_a); X's scale from its maximum (nfi_absmax_slots), or from `slots`
    the producer of X already filled (e.g. nfi_syn_up_conv_act_backward_max; the GEMM clears them)."""
    hi, lo, inv = As
    X = X.contiguous()
    B, K, N = X.shape
    Mrows = hi.shape[1]
    assert hi.shape[2] == K, (hi.shape, X.shape)
    st = _stream(X.device)
    if slots is None:
        slots = torch.empty((slot_words(),), device=X.device, dtype=torch.int32)   # per-image maxima + counter
        _call('nfi_absmax_slots', _p(X), B, K * N, _p(slots), st)
    C = torch.empty((B, Mrows, N), device=X.device)
    ks = ksplit(B * -(-Mrows // 128) * -(-N // 128), K) if (Mrows * N) % 4 == 0 else 1
    work = torch.empty((ks, B, Mrows, N), device=X.device) if ks > 1 else None
    _call('nfi_gemm_split16_shared_a', _p(hi), _p(lo), _p(inv), _p(X), _p(slots), _p(C), B, Mrows, N, K, ks,
          _p(work), st)
    return C


def ksplit(tiles, K):
    """K ranges for a split GEMM of `tiles` 128 x 128 output tiles: enough workgroups to cover the
    256 CUs about twice (each range at least 8 K-steps of 32)."""
    if tiles >= 512:
        return 1
    return max(1, min(K // 256, -(-512 // tiles)))


def stream_slots(owner: dict, device):
    """A self-clearing maxima buffer (per-image slots + the GEMM's counter, zeroed once) per stream, kept in
    `owner` — for producers that fill the maxima of a split product's B operand themselves."""
    key = torch.cuda.current_stream(device).cuda_stream
    buf = owner.get(key)
    if buf is None:
        buf = owner[key] = torch.zeros((slot_words(),), device=device, dtype=torch.int32)
    return buf


def _slots(Uw: WeightSet, device):
    """The maxima slots of this layer's split products on the current stream: per-image running maxima +
    a completion counter, zeroed once; the input transform fills them and the GEMM's last workgroup
    returns them to zero (include/nfi_producer.h), so no memset per call.  One buffer per stream: the
    LPIPS target features run the same layers on a side stream."""
    key = torch.cuda.current_stream(device).cuda_stream
    buf = Uw.vmax.get(key)
    if buf is None:
        buf = Uw.vmax[key] = torch.zeros((slot_words(),), device=device, dtype=torch.int32)
    return buf


def _product(Uw: WeightSet, x, scale=None, relu_y=None):
    """Input transform of x [N, K, H, W] (times scale [N, K]; through the ReLU mask of relu_y) and
    the 36 products with the transformed weights: M [36, Mrows, P]."""
    N, K, H, W = x.shape
    P = N * (H // 4) * (W // 4)
    st = _stream(x.device)
    V = torch.empty((36, K, P), device=x.device)
    if SPLIT16 and Uw.split is not None:
        hi, lo, inv = Uw.split
        vmax = _slots(Uw, x.device)
        _call('nfi_wino_input_transform_max', _p(x), _p(scale), _p(relu_y), _p(V), _p(vmax), N, K, H, W, st)
        Mrows = Uw.U.shape[1]
        M = torch.empty((36, Mrows, P), device=x.device)
        ks = ksplit(36 * -(-Mrows // 128) * -(-P // 128), K) if KSPLIT and (Mrows * P) % 4 == 0 else 1
        if ks > 1:
            work = torch.empty((ks, 36, Mrows, P), device=x.device)
            _call('nfi_gemm_split16_ksplit', _p(hi), _p(lo), _p(inv), _p(V), _p(vmax), _p(M), 36, Mrows, P, K, P // N,
                  ks, _p(work), st)
        else:
            _call('nfi_gemm_split16', _p(hi), _p(lo), _p(inv), _p(V), _p(vmax), _p(M), 36, Mrows, P, K, P // N, st)
        return M
    if relu_y is not None:
        _call('nfi_wino_input_transform_relu_grad', _p(x), _p(relu_y), _p(V), N, K, H, W, st)
    else:
        _call('nfi_wino_input_transform_scaled', _p(x), _p(scale), _p(V), N, K, H, W, st)
    return torch.bmm(Uw.U, V)


def _pack(U, Co, Ci, st):
    if Ci % 8:
        return None
    lib = _lib.load()
    Ua = torch.empty((int(lib.nfi_wino_packed_size(Co, Ci)),), device=U.device)
    _call('nfi_wino_pack_weights', _p(U), _p(Ua), Co, Ci, st)
    return Ua


def _winograd(x, Uw, bias=None, pool=False, scale=None):
    """x [N,Ci,H,W] (contiguous) with transformed weights Uw = (U [36,Co,Ci], packed or None) ->
    y [N,Co,H,W] (and the pooled map when pool).  scale [N,Ci]: convolve x * scale[n, c]
    (three-pass form: folded into the input transform)."""
    U, Ua = Uw.U, Uw.packed
    N, Ci, H, W = x.shape
    Co = U.shape[1]
    st = _stream(x.device)
    y = torch.empty((N, Co, H, W), device=x.device)
    m = torch.empty((N, Co, H // 2, W // 2), device=x.device) if pool else None
    fused = _fused_ok(Uw, Ci, Co)
    if scale is not None and fused:
        x = x * scale[:, :, None, None]          # (the fused kernel takes no scale)
        scale = None
    if fused:
        if FUSED_SPLIT and Uw.split is not None and Co % 64 == 0 and H % 16 == 0 and W % 16 == 0:
            hi, lo, inv = Uw.split
            _call('nfi_wino_conv_fused_split', _p(x), _p(hi), _p(lo), _p(inv), _p(bias), _p(y), _p(m), N, Ci, Co,
                  H, W, st)
        else:
            _call('nfi_wino_conv_fused', _p(x), _p(Ua), _p(bias), _p(y), _p(m), N, Ci, Co, H, W, st)
        return (y, m) if pool else y
    M = _product(Uw, x, scale)
    _call('nfi_wino_output_transform', _p(M), _p(bias), _p(y), _p(m), N, Co, H, W, st)
    return (y, m) if pool else y


def _dgrad(g, ctx):
    if DGRAD:
        return _conv(g, ctx.Ut)
    return torch.nn.grad.conv2d_input(ctx.xshape, ctx.weight, g, 1, 1)


def _frozen_weight(*ts):
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts):
        raise NotImplementedError('nfi.conv: convolution weights are frozen in the inversion path '
                                  '(no weight gradient); call requires_grad_(False) on the module')


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        _require_device(x, weight)
        x = x.contiguous()
        U, Ut = weights(weight)
        ctx.Ut, ctx.xshape, ctx.weight = Ut, x.shape, weight.detach()
        return _conv(x, U)

    @staticmethod
    def backward(ctx, g):
        return _dgrad(g.contiguous(), ctx), None


class _ModConv(torch.autograd.Function):
    """conv2d(x * s[:, :, None, None], w, padding=1): the modulated convolution of a synthesis
    layer (stylegan.py:130-133 with the weight shared over the batch), the modulation folded into
    the Winograd input transform.  Backward: the data-gradient Winograd, then d x = g' s and
    d s = sum_hw g' x in one pass (nfi_syn_scale_backward)."""

    @staticmethod
    def forward(ctx, x, s, weight):
        _require_device(x, s, weight)
        x = x.contiguous()
        s = s.contiguous()
        U, Ut = weights(weight)
        ctx.save_for_backward(x, s)
        ctx.Ut, ctx.xshape, ctx.weight = Ut, x.shape, weight.detach()
        return _conv(x, U, scale=s)

    @staticmethod
    def backward(ctx, g):
        x, s = ctx.saved_tensors
        g = g.contiguous()
        B, C, H, W = x.shape
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ds = torch.empty((B, C), device=x.device, dtype=x.dtype)
        st = _stream(x.device)
        Co = g.shape[1]
        if DGRAD and DIRECT_MOD and _direct_ok(ctx.Ut, g):
            # the data gradient on the direct kernel, then gx = g' s and ds = sum_hw g' x in one pass
            gxs = _direct(g, ctx.Ut)
            _call('nfi_syn_scale_backward', _p(gxs), _p(x), _p(s), _p(gx), _p(ds), B * C, H * W, st)
            return gx, ds, None
        if DGRAD and not _fused_ok(ctx.Ut, Co, C):
            # three-pass data gradient, the scale backward in its output transform
            M = _product(ctx.Ut, g)
            _call('nfi_wino_output_transform_scaled_grad', _p(M), _p(x), _p(s), _p(gx), _p(ds), B, C, H, W, st)
            return gx, ds, None
        gxs = _dgrad(g, ctx)
        _call('nfi_syn_scale_backward', _p(gxs), _p(x), _p(s), _p(gx), _p(ds), B * C, H * W, st)
        return gx, ds, None


class _VggBlock(torch.autograd.Function):
    """relu(conv2d(x, w, padding=1) + b) (+ MaxPool2d(2, 2)) with the epilogue in the output
    transform; backward: nfi_vgg_relu_backward, then the data-gradient Winograd."""

    @staticmethod
    def forward(ctx, x, weight, bias, pool: bool):
        _require_device(x, weight, bias)
        x = x.contiguous()
        U, Ut = weights(weight)
        r = _conv(x, U, bias.detach().contiguous(), pool)
        y = r[0] if pool else r
        ctx.save_for_backward(y)
        ctx.Ut, ctx.xshape, ctx.weight = Ut, x.shape, weight.detach()
        ctx.set_materialize_grads(False)
        return r

    @staticmethod
    def backward(ctx, gy, gm=None):
        y, = ctx.saved_tensors
        if gy is None and gm is None:
            return None, None, None, None
        N, C, H, W = y.shape
        gy = None if gy is None else gy.contiguous()
        gm = None if gm is None else gm.contiguous()
        if gm is None and DGRAD and _direct_ok(ctx.Ut, y):
            # no pool gradient: the ReLU threshold inside the direct kernel's staging
            return _direct(gy, ctx.Ut, relu_y=y), None, None, None
        if RELU_IN_TRANSFORM and gm is None and DGRAD and not _fused_ok(ctx.Ut, C, ctx.Ut.U.shape[1]):
            # no pool gradient: the ReLU threshold inside the data gradient's input transform
            st = _stream(y.device)
            M = _product(ctx.Ut, gy, relu_y=y)
            Ci = ctx.Ut.U.shape[1]
            gx = torch.empty((N, Ci, H, W), device=y.device)
            _call('nfi_wino_output_transform', _p(M), None, _p(gx), None, N, Ci, H, W, st)
            return gx, None, None, None
        gz = torch.empty_like(y)
        if gm is not None and DGRAD and _direct_ok(ctx.Ut, y):
            # the pool routing + ReLU pass leaves gz's per-image maxima for the direct data gradient
            gmax = torch.zeros((slot_words(),), device=y.device, dtype=torch.int32)
            _call('nfi_vgg_relu_backward_max', _p(gy), _p(gm), _p(y), _p(gz), _p(gmax), N * C, C, H, W,
                  _stream(y.device))
            gz._nfi_absmax = (gmax, gz._version, gz.data_ptr())
        else:
            _call('nfi_vgg_relu_backward', _p(gy), _p(gm), _p(y), _p(gz), N * C, H, W, _stream(y.device))
        return _dgrad(gz, ctx), None, None, None


def conv3x3(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """F.conv2d(x, weight, padding=1) (no bias): Winograd when applicable and the weight is
    frozen; MIOpen otherwise (other shapes, or a weight that is being trained)."""
    if not applicable(x, weight) or weight.requires_grad:
        return F.conv2d(x, weight, None, 1, 1)
    return _Conv.apply(x, weight)


def modulated_conv3x3(x: torch.Tensor, s: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """F.conv2d(x * s[:, :, None, None], weight, padding=1) for a frozen weight (the synthesis
    layers' modulation, stylegan.py:130); Winograd with the scale folded in when applicable."""
    if not FOLD_SCALE or not applicable(x, weight) or weight.requires_grad:
        from .producer_ops import scale as _scale
        return conv3x3(_scale(x, s), weight)
    return _ModConv.apply(x, s, weight)


def vgg_block(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, pool: bool):
    """relu(conv2d(x, weight, bias, padding=1)) and, when pool, also MaxPool2d(2, 2) of it:
    (y, pooled).  Requires applicable(x, weight)."""
    _frozen_weight(weight, bias)
    return _VggBlock.apply(x, weight, bias, pool)
