"""CPU ORACLE for the caller side of the inversion step — TEST INFRASTRUCTURE ONLY.

The reference's op sequence for the tri-plane producer (StyleGAN2 synthesis network,
models/stylegan.py:293-490, and the AttentionMapper, models/generator.py:42-60, 132-186) and
for the LPIPS-VGG distance (lib/metrics.py:104-146 around `lpips` 0.1, third-party and absent
here: its published algorithm) restated in plain PyTorch over the PARAMETERS of nfi's modules
(nfi.producer.InversionGenerator, nfi.lpips.LPIPS — same state_dict keys as the reference's), on
any device.  nfi itself has one implementation of each (the HIP one); this module is what the
tests check it against and what bench.py's cpu_baseline leg times.  Only tests/, smoke() and
bench.py's cpu_baseline may import it.

Pinning: the producer restatement reproduces tests/golden/producer.npz (the reference Generator
at full size with seeded weights, tests/test_producer.py); LPIPS is PARITY UNPINNED (no package,
weights or fixture offline).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

SQRT2 = math.sqrt(2.0)


def _depthwise(x, k, stride: int, transpose: bool):
    """Per-channel 4x4 FIR with padding 1 (stylegan.py EfficientResample)."""
    b, c, h, w = x.shape
    xf = x.reshape(b * c, 1, h, w)
    kk = k[None, None].to(x.dtype)
    y = (F.conv_transpose2d(xf, kk, padding=1, stride=stride) if transpose
         else F.conv2d(xf, kk, padding=1, stride=stride))
    return y.reshape(b, c, y.shape[-2], y.shape[-1])


def modulated_conv(m, x, w):
    """SynthesisLayer (stylegan.py:293-360, conv_modulated2d :114-145): modulated 3x3 conv with
    demodulation, optional 2x up-sampling (transposed conv + FIR), bias, sqrt(2) gain, leaky ReLU."""
    styles = m.affine(w)                                           # [b, in]
    wmod = m.weight[None] * styles[:, None, :, None, None]         # [b, out, in, 3, 3]
    dcoefs = (wmod.square().sum(dim=(2, 3, 4)) + 1e-8).rsqrt()     # [b, out]
    x = x * styles[:, :, None, None]
    if m.up:
        x = F.conv_transpose2d(x, m.weight.transpose(0, 1), stride=2)
        x = _depthwise(x, m.resample_filter * 4, stride=1, transpose=False)
    else:
        x = F.conv2d(x, m.weight, padding=1)
    x = x * dcoefs[:, :, None, None]
    x = (x + m.bias[None, :, None, None]) * SQRT2
    return F.leaky_relu(x, 0.2)


def to_planes(m, x, w):
    """OutputLayer (stylegan.py:363-384): modulated 1x1 conv, no demodulation, plus bias."""
    styles = m.affine(w) * m.weight_gain
    return F.conv2d(x * styles[:, :, None, None], m.weight) + m.bias[None, :, None, None]


def synthesis(net, ws):
    """SynthesisNetwork.forward (stylegan.py:449-490): blocks at 4 .. res, skip images summed
    through the 2x FIR up-sampling (upsample2d, gain 4)."""
    rows = ws.unbind(1)
    x = img = None
    k = 0
    for r in net.resolutions:
        blk = getattr(net, f'b{r}')
        ws_b = rows[k:k + blk.num_conv + 1]
        j = 0
        if blk.in_ch == 0:
            x = blk.const[None].expand(ws_b[0].shape[0], -1, -1, -1)
        else:
            x = modulated_conv(blk.conv0, x, ws_b[j])
            j += 1
        x = modulated_conv(blk.conv1, x, ws_b[j])
        y = to_planes(blk.torgb, x, ws_b[j + 1])
        img = y if img is None else _depthwise(img, blk.resample_filter * 4, stride=2, transpose=True) + y
        k += blk.num_conv
    return img


def palette(mapper, c):
    """AttentionMapper.forward (generator.py:166-186) with ConditionalLayerNorm (:42-60)."""
    scale = SQRT2 / 2
    x = mapper.const.expand(c.shape[0], -1)
    for pair in ((1, 2), (3, 4)):
        shortcut = x
        for i in pair:
            h = getattr(mapper, f'fc{i}')(x)
            n = getattr(mapper, f'norm{i}')
            h = torch.addcmul(n.fc_beta(c), 1 + n.fc_gamma(c), F.layer_norm(h, (n.ch,)))
            x = F.leaky_relu(h, 0.2)
        x = (x + shortcut) * scale
    x = F.leaky_relu(mapper.fc5(x), 0.2)
    return torch.sigmoid(mapper.fc_values(x).view(-1, mapper.num_values, 3)) * 2.004 - 1.002


def planes_and_palette(gen, ws):
    """Generator.forward's producer half (generator.py:451-477): ws [b,15,512] -> planes
    [b,3,32,R,R] and the palette [b,10,3]."""
    w_syn, w_tex = ws.split([14, ws.shape[1] - 14], dim=1)
    pal = palette(gen.texture_mapper, w_tex[:, 0])
    planes = synthesis(gen.synthesis_network, w_syn)
    return planes.view(ws.shape[0], 3, 32, planes.shape[-2], planes.shape[-1]), pal


class ReferenceProducer:
    """An nfi.producer.InversionGenerator whose planes_and_palette is the reference's op sequence
    (everything else — decoder, alpha, beta, mapping network, state_dict — is the wrapped
    generator's): the CPU inversion loop of the tests and of bench.py's cpu_baseline."""

    def __init__(self, gen):
        object.__setattr__(self, 'gen', gen)

    def planes_and_palette(self, ws):
        return planes_and_palette(self.gen, ws)

    def __getattr__(self, name):
        return getattr(self.gen, name)


# ---------------------------------------------------------------------------------------------
# LPIPS (lpips 0.1, LPIPS(net='vgg'); lib/metrics.py:104-146)

def lpips_features(net, im):
    """ScalingLayer then torchvision VGG16 features cut after relu1_2 .. relu5_3."""
    from nfi.lpips import TAPS
    x = (im - net.shift) / net.scale
    out = []
    for i, layer in enumerate(net.net.features):
        x = layer(x)
        if i in TAPS:
            out.append(x)
    return out


def lpips_normalize(x):
    """lpips.normalize_tensor (eps 1e-10)."""
    return x / (x.square().sum(dim=1, keepdim=True).sqrt() + 1e-10)


def lpips_distance(net, in0, in1=None, f1=None):
    """sum_l mean_hw(lin_l((n(f0_l) - n(f1_l))^2)) -> [N, 1], over nfi.lpips.LPIPS's parameters."""
    f0 = lpips_features(net, in0)
    if f1 is None:
        f1 = lpips_features(net, in1)
    return sum(lin((lpips_normalize(a) - lpips_normalize(b)).square()).mean(dim=[2, 3])
               for a, b, lin in zip(f0, f1, net.lins))


class ReferenceLPIPS:
    """nfi.lpips.LPIPS's interface (forward, target_features) over the reference op sequence."""

    def __init__(self, net):
        self.net = net

    def target_features(self, in1):
        with torch.no_grad():
            return lpips_features(self.net, in1)

    def __call__(self, in0, in1=None, f1=None):
        return lpips_distance(self.net, in0, in1, f1)
