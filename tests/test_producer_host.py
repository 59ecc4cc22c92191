"""Host-side logic of the producer's HIP path that runs without a GPU: the style bank's packed
per-layer views (one gather forward, one scatter backward) and the strided-layout descriptors of
the skip-image chain (channels-last / texel-major planes)."""

import torch
from torch import nn

from nfi import producer, producer_ops


def test_pack_rows_forward_and_backward():
    torch.manual_seed(0)
    L, b, W = 4, 3, 8
    widths = [8, 5, 8, 2]
    X = torch.randn(L, b, W, dtype=torch.float32, requires_grad=True)
    holder = nn.Module()
    idx = producer._pack_index(holder, 'k', X.shape, widths, X.device)
    assert producer._pack_index(holder, 'k', X.shape, widths, X.device) is idx      # cached
    outs = producer._PackRows.apply(X, idx, b, widths)
    for l, (o, n) in enumerate(zip(outs, widths)):
        assert o.shape == (b, n) and o.is_contiguous()
        assert torch.equal(o, X[l, :, :n])
    gs = [torch.randn(b, n) for n in widths]
    torch.autograd.backward(list(outs), gs)
    ref = torch.zeros(L, b, W)
    for l, (g, n) in enumerate(zip(gs, widths)):
        ref[l, :, :n] = g
    assert torch.equal(X.grad, ref)


def test_pack_rows_unused_outputs_get_zero_gradient():
    X = torch.randn(2, 2, 4, requires_grad=True)
    widths = [3, 4]
    idx = producer._pack_index(nn.Module(), 'k', X.shape, widths, X.device)
    outs = producer._PackRows.apply(X, idx, 2, widths)
    outs[1].sum().backward()                    # outs[0] takes no gradient
    ref = torch.zeros(2, 2, 4)
    ref[1] = 1.0
    assert torch.equal(X.grad, ref)


def test_layout_descriptors():
    B, C, h, w = 2, 96, 8, 12
    cl = torch.empty(B, C, h, w).to(memory_format=torch.channels_last)
    s = producer_ops._str3(cl)
    assert tuple(s) == (h * w * C, 32, C)
    planes = producer_ops._texel_major((B, 3, 32, h, w), 'cpu', torch.float32)
    s = producer_ops._str3(planes)
    assert tuple(s) == (3 * h * w * 32, h * w * 32, 32)
    assert planes.permute(0, 1, 3, 4, 2).is_contiguous()
    nchw = torch.empty(B, C, h, w)
    assert producer_ops._str3(nchw) is None
    assert producer_ops._str3(producer_ops._conform(nchw)) is not None
    p5 = torch.empty(B, 3, 32, h, w)                       # channel-major 5-d: conformed by a copy
    assert producer_ops._str3(p5) is None
    assert producer_ops._str3(producer_ops._conform(p5)) is not None
