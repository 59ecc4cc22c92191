"""Strided producer outputs as planes: a dense channels_last buffer is used as a
texel-major view without a copy; batch-sliced and channel-sliced channels_last buffers are not
dense and take the copy path.  Every form must give the outputs and gradients of the contiguous
planes (d planes up to float-atomic summation order)."""

import pytest
import torch

import nfi
from gpu_helpers import rel_l2, synthetic_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _render(inp, meta, planes):
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False, fine_sampling=True)
    f = nfi.TriplaneField(planes=planes, palette=inp['palette'].to(DEV), w1=inp['w1'].to(DEV),
                          b1=inp['b1'].to(DEV), w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0,
                          beta=0.1)
    rgb, depth, mask, _, _, _ = nfi.render(f, meta['H'], meta['W'], inp['cam'].to(DEV), inp['focal'].to(DEV),
                                           None, None, None, meta['S'], randomize=True,
                                           u_coarse=inp['u_coarse'].to(DEV), u_fine=inp['u_fine'].to(DEV))
    loss = (rgb * inp['g_rgb'].to(DEV)).sum() + (mask * inp['g_mask'].to(DEV)).sum()
    return rgb.detach(), mask.detach(), loss


@pytest.mark.parametrize('form', ['channels_last', 'batch_strided', 'channel_sliced'])
def test_strided_planes(form):
    inp, meta = synthetic_inputs(B=2, H=16, W=16, S=16, R=32, scene_range=1.4, seed=21)
    B, R = 2, 32
    base = inp['planes'].to(DEV).reshape(B, 96, R, R)
    ref_leaf = base.clone().requires_grad_()
    r_rgb, r_mask, r_loss = _render(inp, meta, ref_leaf.view(B, 3, 32, R, R))
    r_loss.backward()
    if form == 'channels_last':
        buf = base.clone().to(memory_format=torch.channels_last)
        leaf = buf.requires_grad_()
        planes_in = leaf
    elif form == 'batch_strided':
        buf = torch.zeros(2 * B, 96, R, R, device=DEV).to(memory_format=torch.channels_last)
        buf[::2] = base
        leaf = buf.requires_grad_()
        planes_in = leaf[::2]
    else:
        buf = torch.zeros(B, 128, R, R, device=DEV).to(memory_format=torch.channels_last)
        buf[:, :96] = base
        leaf = buf.requires_grad_()
        planes_in = leaf[:, :96]
    rgb, mask, loss = _render(inp, meta, planes_in.view(B, 3, 32, R, R))
    loss.backward()
    assert torch.equal(rgb, r_rgb) and torch.equal(mask, r_mask)
    g = leaf.grad
    g = {'channels_last': g, 'batch_strided': g[::2], 'channel_sliced': g[:, :96]}[form]
    assert rel_l2(g, ref_leaf.grad) < 1e-5
    if form == 'batch_strided':
        assert float(leaf.grad[1::2].abs().max()) == 0.0
    if form == 'channel_sliced':
        assert float(leaf.grad[:, 96:].abs().max()) == 0.0
