"""LPIPS-VGG (nfi/lpips.py).  PARITY UNPINNED: the reference calls the
third-party `lpips` 0.1 package with pretrained VGG16 + lin weights (lib/metrics.py:104-146);
neither the package nor the weights exist offline, so no reference output can be produced.
These CPU tests check the restated structure: state_dict layout of the two weight files it
loads, the metric's identities (d(x, x) = 0, symmetry, non-negativity), and the distance head
against a direct per-pixel evaluation — on the oracle's PyTorch formulation over the module's
parameters (oracle/producer_oracle.py: nfi.lpips itself runs on the GPU only).  The HIP LPIPS is
checked against it in tests/test_gpu_lpips.py."""

import pytest
import torch

from nfi import lpips
from oracle import producer_oracle as po


def test_weight_layout_matches_torchvision_and_lpips_files():
    net = lpips.LPIPS()
    keys = set(net.net.state_dict())
    # torchvision vgg16().features conv indices
    convs = [0, 2, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28]
    assert keys == {f'features.{i}.{p}' for i in convs for p in ('weight', 'bias')}
    vgg_sd = {k: torch.randn_like(v) for k, v in net.net.state_dict().items()}
    vgg_sd['classifier.0.weight'] = torch.zeros(1)       # ignored
    lin_sd = {f'lin{i}.model.1.weight': torch.rand(1, c, 1, 1) for i, c in enumerate(lpips.CHANNELS)}
    net.load_weights(vgg_sd, lin_sd)
    assert torch.equal(net.net.features[28].weight, vgg_sd['features.28.weight'])
    assert torch.equal(net.lins[3].weight, lin_sd['lin3.model.1.weight'])


def test_metric_identities():
    torch.manual_seed(0)
    net = po.ReferenceLPIPS(lpips.LPIPS())
    a = torch.tanh(torch.randn(3, 3, 64, 64))
    b = torch.tanh(torch.randn(3, 3, 64, 64))
    dab, dba, daa = net(a, b), net(b, a), net(a, a)
    assert dab.shape == (3, 1)
    assert torch.all(dab > 0)
    torch.testing.assert_close(dab, dba, rtol=1e-5, atol=1e-7)
    assert float(daa.abs().max()) == 0.0


def test_distance_head_per_pixel():
    torch.manual_seed(1)
    f0, f1 = torch.randn(2, 5, 3, 4).relu(), torch.randn(2, 5, 3, 4).relu()
    w = torch.rand(5)
    got = (po.lpips_normalize(f0) - po.lpips_normalize(f1)).square().mul(w[None, :, None, None]).sum(1).mean((1, 2))
    want = torch.zeros(2)
    for n in range(2):
        for y in range(3):
            for x in range(4):
                a, b = f0[n, :, y, x], f1[n, :, y, x]
                na, nb = a / (a.norm() + 1e-10), b / (b.norm() + 1e-10)
                want[n] += (w * (na - nb) ** 2).sum() / 12
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize('white', [False, True])
def test_vgg_loss_matches_reference_augmentation_order(white):
    """image_loss('vgg') samples the prediction and target copies separately with one grid; the
    reference (run.py:2214-2235) augments cat((pred, target), channels) — same loss, and the same
    gradient to the prediction."""
    from nfi import inversion
    torch.manual_seed(3)
    net = po.ReferenceLPIPS(lpips.LPIPS())
    rgb = torch.tanh(torch.randn(2, 32, 32, 3)).requires_grad_()
    target = torch.tanh(torch.randn(2, 32, 32, 3))
    got = inversion.image_loss('vgg', rgb, target, net, white, torch.Generator().manual_seed(5))
    got.backward()
    g_got = rgb.grad.clone()
    rgb.grad = None
    pred, tgt = rgb.permute(0, 3, 1, 2), target.permute(0, 3, 1, 2)
    cat = torch.cat((pred, tgt), dim=1).unsqueeze(1).expand(-1, 15, -1, -1, -1).contiguous().flatten(0, 1)
    cat = inversion.augment_images(cat, 1.0, white, generator=torch.Generator().manual_seed(5))
    want = net(torch.cat((pred, cat[:, :3])), torch.cat((tgt, cat[:, 3:]))).mean() * 2
    want.backward()
    assert torch.equal(got.detach(), want.detach())
    torch.testing.assert_close(g_got, rgb.grad, rtol=1e-6, atol=1e-9)
