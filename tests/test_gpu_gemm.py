"""The split-f16 batched GEMM (csrc/nfi_gemm.hip, nfi_gemm_split16) against fp64: C[b] = A[b] B[b]
with fp32 operands carried as power-of-two-scaled hi + lo fp16 pairs on the f16 matrix cores
(three products each).  Bound: the fp64-relative error of each batch entry within 4x of the fp32
GEMM's own (torch.bmm on the device, hipBLASLt) plus a floor of 2^-22 of the entry's |A||B| scale;
partial M / N tiles, K from 32 to 512, operands spanning magnitudes across the batch."""

import ctypes

import pytest
import torch

from nfi import _lib, conv

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def split_gemm(A, B):
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    b, M, K = A.shape
    N = B.shape[2]
    hi = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    lo = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    inv = torch.empty((b,), device=DEV)
    _lib.check(lib.nfi_split16_pack(_p(A), b, M * K, _p(hi), _p(lo), _p(inv), st), 'nfi_split16_pack')
    slots = torch.empty((conv.slot_words(),), device=DEV, dtype=torch.int32)   # per-image maxima + counter
    _lib.check(lib.nfi_absmax_slots(_p(B), 1, B.numel(), _p(slots), st), 'nfi_absmax_slots')
    C = torch.empty((b, M, N), device=DEV)
    _lib.check(lib.nfi_gemm_split16(_p(hi), _p(lo), _p(inv), _p(B), _p(slots), _p(C), b, M, N, K, N, st),
               'nfi_gemm_split16')
    return C


@pytest.mark.parametrize('b,M,N,K', [(4, 64, 1000, 64), (36, 128, 4096, 128), (3, 96, 257, 32), (2, 512, 1024, 512),
                                     (36, 256, 300, 256), (5, 160, 516, 96), (2, 200, 132, 32)])
def test_split16_gemm_matches_fp64(b, M, N, K):
    """One image per call (cols_per_image = N): B's scale is one for the call, A's per batch entry."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn((b, M, K), device=DEV, generator=g)
    B = torch.randn((b, K, N), device=DEV, generator=g)
    # magnitudes spread across the batch entries (A's scale is per entry, B's per call)
    A *= torch.logspace(-3, 3, b, device=DEV)[:, None, None]
    B *= torch.logspace(2, -2, b, device=DEV)[:, None, None]
    C = split_gemm(A, B)
    ref64 = torch.bmm(A.double(), B.double())
    ref32 = torch.bmm(A, B)
    for i in range(b):
        scale = float((A[i].double().abs() @ B[i].double().abs()).max())
        e_hip = float((C[i].double() - ref64[i]).abs().max()) / scale
        e_ref = float((ref32[i].double() - ref64[i]).abs().max()) / scale
        assert e_hip <= 4 * e_ref + 2 ** -22, (i, e_hip, e_ref)


@pytest.mark.parametrize('Ci,Co,H', [(128, 128, 32), (256, 512, 16), (128, 64, 64), (512, 512, 16), (512, 512, 8)])
def test_winograd_split16_matches_bmm(Ci, Co, H):
    """The three-pass Winograd convolution with the split-f16 products against the same pipeline with
    hipBLASLt's fp32 bmm, and both against an fp64 direct convolution (the 2e-5 bound of
    tests/test_gpu_conv.py).  512 -> 512 at 16^2 / 8^2: few output tiles, K split in two
    (nfi_gemm_split16_ksplit)."""
    g = torch.Generator(device=DEV).manual_seed(Ci + Co)
    x = torch.randn((4, Ci, H, H), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    Uw, _ = conv.weights(w)
    assert Uw.split is not None
    old = conv.FUSED, conv.SPLIT16
    out = {}
    try:
        conv.FUSED = False
        for mode in (True, False):
            conv.SPLIT16 = mode
            out[mode] = conv._winograd(x, Uw)
    finally:
        conv.FUSED, conv.SPLIT16 = old
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
    scale = float(ref.abs().max())
    e_split = float((out[True].double() - ref).abs().max()) / scale
    e_bmm = float((out[False].double() - ref).abs().max()) / scale
    print(f'  split16 {e_split:.3g}  bmm {e_bmm:.3g}')
    assert e_split <= 2e-5 and e_split <= 2 * e_bmm + 1e-6


@pytest.mark.parametrize('b,M,N,K', [(4, 9 * 64, 256, 128), (2, 9 * 32, 1024, 96), (3, 64, 36, 4608),
                                     (4, 512, 64, 4608), (2, 256, 1000, 1152)])
def test_split16_shared_a_matches_fp64(b, M, N, K):
    """nfi_gemm_split16_shared_a (conv.split_matmul_shared): one A for every batch entry — the
    up-sampling convolutions' 9-tap matrix W9 [9 Co, Ci] against each image, and W9^T [Ci, 9 Co]
    against the tap gradients (K = 9 Co; few output tiles: K split in ranges, conv.ksplit)."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 1)
    A = torch.randn((M, K), device=DEV, generator=g) * 1e-2
    X = torch.randn((b, K, N), device=DEV, generator=g) * torch.logspace(1, -1, b, device=DEV)[:, None, None]
    old = conv.SPLIT16
    try:
        conv.SPLIT16 = True
        C = conv.split_matmul_shared(conv.split_matrix(A), X)
    finally:
        conv.SPLIT16 = old
    ref64 = torch.matmul(A.double(), X.double())
    ref32 = torch.matmul(A, X)
    for i in range(b):
        scale = float((A.double().abs() @ X[i].double().abs()).max())
        e_hip = float((C[i].double() - ref64[i]).abs().max()) / scale
        e_ref = float((ref32[i].double() - ref64[i]).abs().max()) / scale
        assert e_hip <= 4 * e_ref + 2 ** -22, (i, e_hip, e_ref)


def test_maxima_slots_back_to_back_and_after_rejection():
    """The split product's self-clearing maxima slots (nfi_gemm.hip release_slots: the input transform
    fills the per-image running maxima, the GEMM's last workgroup returns them to zero).  (1) One layer's
    three-pass Winograd convolution back to back on inputs whose maxima shrink by 2^10 and 2^20 and
    grow back: each call within the fp64 bound on its OWN scale (a slot still holding the previous
    call's larger maximum would coarsen the next B scale by that factor).  (2) The input transform
    fills the slots from a large input, then the GEMM call is rejected (K not a multiple of 32): the
    rejection zeroes the slots, so the next call on an input 2^30 smaller keeps its precision (a stale
    maximum would put its operands 2^30 below the scale: fp16 underflow, error ~1)."""
    g = torch.Generator(device=DEV).manual_seed(7)
    Ci, Co, H = 64, 128, 32
    x = torch.randn((2, Ci, H, H), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    Uw, _ = conv.weights(w)
    assert Uw.split is not None

    def check(xs):
        y = conv._winograd(xs, Uw)
        ref = torch.nn.functional.conv2d(xs.double(), w.double(), padding=1)
        e = float((y.double() - ref).abs().max() / ref.abs().max())
        assert e <= 2e-5, e

    old = conv.FUSED, conv.SPLIT16
    try:
        conv.FUSED, conv.SPLIT16 = False, True
        for s in (1.0, 2.0 ** -10, 2.0 ** -20, 1.0):
            check(x * s)
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
        vmax = conv._slots(Uw, DEV)
        P = 2 * (H // 4) * (H // 4)
        V = torch.empty((36, Ci, P), device=DEV)
        big = x * 2.0 ** 10
        _lib.check(lib.nfi_wino_input_transform_max(_p(big), None, None, _p(V), _p(vmax), 2, Ci, H, H, st),
                   'nfi_wino_input_transform_max')
        assert int(vmax[:-1].abs().sum()) > 0
        hi, lo, inv = Uw.split
        M = torch.empty((36, Co, P), device=DEV)
        rc = lib.nfi_gemm_split16(_p(hi), _p(lo), _p(inv), _p(V), _p(vmax), _p(M), 36, Co, P, Ci + 1, P // 2, st)
        assert rc != 0, 'K % 32 != 0 must be rejected'
        torch.cuda.synchronize()
        assert int(vmax.abs().sum()) == 0, 'a rejected call must leave the maxima slots zeroed'
        check(x * 2.0 ** -20)
    finally:
        conv.FUSED, conv.SPLIT16 = old


@pytest.mark.parametrize('K,ks', [(160, 4), (96, 3), (224, 5)])
def test_ksplit_ranges_never_empty(K, ks):
    """nfi_gemm_split16_ksplit with a split the K steps do not fill evenly (K = 160 = 5 steps in 4
    ranges used to leave range 3 empty and load past the operands): the ranges are re-cut so that none
    is empty, and the result stays within the fp64 bound."""
    g = torch.Generator(device=DEV).manual_seed(K + ks)
    b, M, N = 3, 96, 200
    A = torch.randn((b, M, K), device=DEV, generator=g)
    B = torch.randn((b, K, N), device=DEV, generator=g)
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    hi = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    lo = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    inv = torch.empty((b,), device=DEV)
    _lib.check(lib.nfi_split16_pack(_p(A), b, M * K, _p(hi), _p(lo), _p(inv), st), 'nfi_split16_pack')
    slots = torch.empty((conv.slot_words(),), device=DEV, dtype=torch.int32)
    _lib.check(lib.nfi_absmax_slots(_p(B), 1, B.numel(), _p(slots), st), 'nfi_absmax_slots')
    C = torch.empty((b, M, N), device=DEV)
    work = torch.empty((ks, b, M, N), device=DEV)
    _lib.check(lib.nfi_gemm_split16_ksplit(_p(hi), _p(lo), _p(inv), _p(B), _p(slots), _p(C), b, M, N, K, N, ks,
                                           _p(work), st), 'nfi_gemm_split16_ksplit')
    ref64 = torch.bmm(A.double(), B.double())
    ref32 = torch.bmm(A, B)
    for i in range(b):
        scale = float((A[i].double().abs() @ B[i].double().abs()).max())
        e_hip = float((C[i].double() - ref64[i]).abs().max()) / scale
        e_ref = float((ref32[i].double() - ref64[i]).abs().max()) / scale
        assert e_hip <= 4 * e_ref + 2 ** -22, (i, e_hip, e_ref)


def _three_pass(x, w):
    Uw, _ = conv.weights(w)
    old = conv.FUSED, conv.SPLIT16
    try:
        conv.FUSED, conv.SPLIT16 = False, True
        return conv._winograd(x.contiguous(), Uw)
    finally:
        conv.FUSED, conv.SPLIT16 = old


def _rel(a, b, scale):
    return float((a.double() - b.double()).abs().max()) / scale


@pytest.mark.parametrize('small', [1e-6, 1e-9])
@pytest.mark.parametrize('Ci,Co,H', [(128, 128, 32), (256, 256, 16), (512, 512, 8)])
def test_split16_per_image_scale(Ci, Co, H, small):
    """VERDICT r05 item 5 (sharded = unsharded per image).  B's power-of-two scale of the
    split product is per image: a batch of 4 where image 2 sits `small` below the others.  (1) Every
    image, the small one included, within the conv bound (2e-5 of ITS OWN largest output) of an fp64
    convolution.  (2) The small image convolved alone (a shard of one) equals its row of the batch to
    1e-6 of its own scale — with one scale per call it would lose 2^-(39-k) operand precision
    (k = log2(1/small): at 1e-9 the lo halves underflow and the error is ~1e-3 of its scale)."""
    g = torch.Generator(device=DEV).manual_seed(Ci + H)
    x = torch.randn((4, Ci, H, H), device=DEV, generator=g)
    x[2] *= small
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    y = _three_pass(x, w)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
    for i in range(4):
        s = float(ref[i].abs().max())
        e = _rel(y[i], ref[i], s)
        assert e <= 2e-5, (i, e)
    alone = _three_pass(x[2:3], w)
    s2 = float(ref[2].abs().max())
    d = _rel(alone[0], y[2], s2)
    print(f'  small image: fp64 err {_rel(y[2], ref[2], s2):.3g}, alone vs batch {d:.3g}')
    assert d <= 1e-6, d


@pytest.mark.parametrize('small', [1e-6, 1e-9])
def test_split16_shared_a_per_image_scale(small):
    """The shared-A product (up-sampling convolutions: image b = batch entry b): image 2 `small` below
    the others keeps the fp32-GEMM bound on its own scale, and alone equals its row of the batch."""
    g = torch.Generator(device=DEV).manual_seed(11)
    b, M, N, K = 4, 9 * 64, 1024, 128
    A = torch.randn((M, K), device=DEV, generator=g) * 1e-2
    X = torch.randn((b, K, N), device=DEV, generator=g)
    X[2] *= small
    old = conv.SPLIT16
    try:
        conv.SPLIT16 = True
        As = conv.split_matrix(A)
        C = conv.split_matmul_shared(As, X)
        alone = conv.split_matmul_shared(As, X[2:3])
    finally:
        conv.SPLIT16 = old
    ref64 = torch.matmul(A.double(), X.double())
    ref32 = torch.matmul(A, X)
    for i in range(b):
        scale = float((A.double().abs() @ X[i].double().abs()).max())
        e_hip = _rel(C[i], ref64[i], scale)
        e_ref = _rel(ref32[i], ref64[i], scale)
        assert e_hip <= 4 * e_ref + 2 ** -22, (i, e_hip, e_ref)
    s2 = float((A.double().abs() @ X[2].double().abs()).max())
    assert _rel(alone[0], C[2], s2) <= 1e-6


def test_up_conv_backward_per_image_scale():
    """The up-sampling layer's data gradient W9^T dP, whose B maxima come from the fused epilogue
    backward (nfi_syn_up_conv_act_backward_max): one image's output gradient 1e-9 below the others —
    its d x equals the d x of the same image run alone (a shard of one) to 1e-6 of its own scale."""
    from nfi import producer_ops
    g = torch.Generator(device=DEV).manual_seed(5)
    B, Ci, Co, n = 4, 64, 64, 32
    x = torch.randn((B, Ci, n, n), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    d = torch.rand((B, Co), device=DEV, generator=g) + 0.5
    bias = torch.randn((Co,), device=DEV, generator=g) * 0.1
    gy = torch.randn((B, Co, 2 * n, 2 * n), device=DEV, generator=g)
    gy[2] *= 1e-9
    old = conv.SPLIT16
    try:
        conv.SPLIT16 = True

        def dx(xs, ds, gs):
            xs = xs.clone().requires_grad_()
            y = producer_ops.up_conv_act(xs, w, ds.contiguous(), bias, 2 ** 0.5)
            y.backward(gs)
            return xs.grad
        full = dx(x, d, gy)
        alone = dx(x[2:3], d[2:3], gy[2:3])
    finally:
        conv.SPLIT16 = old
    s2 = float(alone.abs().max())
    assert s2 > 0
    e = _rel(alone[0], full[2], s2)
    print(f'  small image d x: alone vs batch {e:.3g}')
    assert e <= 1e-6, e
