"""LPIPS-VGG perceptual loss of the inversion step: lib/metrics.py:104-146
(`LPIPSLoss`, the reference's wrapper) around the third-party `lpips` package, version 0.1
(`lpips.LPIPS(net='vgg')`, its published algorithm restated here — the package and its weights
are not in this image, so PARITY IS UNPINNED for this module: no fixture exists to check it
against, and random weights stand in unless `load_weights` is given the two state_dicts).

  features  ScalingLayer ((x - shift) / scale) then torchvision VGG16 `features` cut after
            relu1_2, relu2_2, relu3_3, relu4_3, relu5_3 (lpips/pretrained_networks.py `vgg16`)
  distance  sum_l mean_hw( lin_l( (n(f0_l) - n(f1_l))^2 ) ), n(x) = x / (||x||_channels + 1e-10),
            lin_l a bias-free 1x1 conv to one channel (lpips/lpips.py NetLinLayer; dropout is
            inactive in eval)

One implementation, on the device: the VGG 3x3 convolutions are Winograd F(4,3) blocks (nfi.conv)
with bias, ReLU and the next 2x2 max pool in their output transform (bias-free MIOpen calls plus
one fused HIP epilogue where Winograd does not apply; the 3-channel first layer one direct HIP
pass); the distance head — normalisation, difference, lin, spatial mean — is one fused HIP kernel
per layer, forward and backward (csrc/nfi_producer.hip).  The op sequence above in plain PyTorch
over this module's parameters is test infrastructure: oracle/producer_oracle.py.
"""

from __future__ import annotations

import ctypes

import os

import torch
import torch.nn.functional as F
from torch import nn

VGG_CFG = [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512]
TAPS = (3, 8, 15, 22, 29)          # torchvision vgg16.features indices of relu1_2 .. relu5_3
CHANNELS = (64, 128, 256, 512, 512)
SHIFT = (-.030, -.088, -.188)      # lpips ScalingLayer
SCALE = (.458, .448, .450)
EPS = 1e-10


class VGG16Features(nn.Module):
    """torchvision.models.vgg16().features[:30] with the same module indices (state_dict keys
    'features.<i>.weight'/'bias' load directly)."""

    winograd = True    # fused path: 3x3 layers as Winograd F(4,3) (nfi.conv) where applicable

    def __init__(self):
        super().__init__()
        layers, c = [], 3
        for v in VGG_CFG:
            if v == 'M':
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=False)]
                c = v
        self.features = nn.Sequential(*layers)

    def forward(self, x, shift=None, scale=None):
        """The feature taps of x; with shift / scale, of the ScalingLayer's (x - shift) / scale, folded
        into the first layer's kernels when they apply (else computed here)."""
        out = []
        from . import producer_ops as _po
        if shift is not None and not (self.winograd and _po.vgg_first_applicable(x, self.features[0].weight)):
            x, shift, scale = (x - shift) / scale, None, None
        # each conv block as MIOpen's bias-free convolution + one HIP epilogue pass (bias, ReLU and
        # the following MaxPool2d when there is one; producer_ops.vgg_epilogue)
        from . import conv as wconv, producer_ops
        f, i = self.features, 0
        while i < len(f):
            conv = f[i]
            pool = i + 2 < len(f) and isinstance(f[i + 2], nn.MaxPool2d)
            if self.winograd and wconv.applicable(x, conv.weight):
                # nfi.conv: the direct split-f16 kernel on the 128^2 / 64^2 maps, Winograd F(4,3)
                # below; the epilogue (bias, ReLU, pool) fused either way
                r = wconv.vgg_block(x, conv.weight, conv.bias, pool)
                y, x = r if pool else (r, r)
                if i + 1 in TAPS:
                    out.append(y)
                i += 3 if pool else 2
                continue
            if i == 0 and not pool and producer_ops.vgg_first_applicable(x, conv.weight):
                x = producer_ops.vgg_first(x, conv.weight, conv.bias, shift, scale)   # (normalise) conv1_1 + ReLU
                if i + 1 in TAPS:
                    out.append(x)
                i += 2
                continue
            z = F.conv2d(x, conv.weight, None, 1, 1)
            if z.shape[-1] % 4 == 0 and not (pool and z.shape[-2] % 2):
                r = producer_ops.vgg_epilogue(z, conv.bias, pool)
                y, x = r if pool else (r, r)
            else:                      # (maps narrower than 4 columns: the unfused ops)
                y = x = F.relu(z + conv.bias[None, :, None, None])
                if pool:
                    x = F.max_pool2d(y, 2, 2)
            if i + 1 in TAPS:
                out.append(y)
            i += 3 if pool else 2
        return out


# the ScalingLayer inside the first VGG layer's kernels (nfi_vgg_first_forward_max / _backward_scaled);
# NFI_LPIPS_FOLD=0: the two ATen ops each way (A/B)
FOLD_SCALING = os.environ.get('NFI_LPIPS_FOLD', '1') != '0'


class LPIPS(nn.Module):
    """`LPIPSLoss` (metrics.py:104-146): forward(in0, in1) -> [N, 1] distances (reduction
    'none'), in0/in1 in [-1, 1] (normalize=False, as run.py:2231 calls it)."""

    def __init__(self):
        super().__init__()
        self.net = VGG16Features()
        self.lins = nn.ModuleList([nn.Conv2d(c, 1, 1, bias=False) for c in CHANNELS])
        self.register_buffer('shift', torch.tensor(SHIFT).view(1, 3, 1, 1))
        self.register_buffer('scale', torch.tensor(SCALE).view(1, 3, 1, 1))
        with torch.no_grad():                  # lpips lin weights are non-negative
            for lin in self.lins:
                lin.weight.abs_().mul_(0.1)
        self.eval()
        self.requires_grad_(False)

    def load_weights(self, vgg_state_dict: dict, lin_state_dict: dict):
        """vgg_state_dict: torchvision vgg16 keys ('features.0.weight', ...); lin_state_dict:
        lpips weights/v0.1/vgg.pth keys ('lin0.model.1.weight', ...).  Load both with
        torch.load(..., weights_only=True)."""
        feats = {k: v for k, v in vgg_state_dict.items() if k.startswith('features.')}
        self.net.load_state_dict(feats, strict=False)
        for i, lin in enumerate(self.lins):
            lin.weight.data.copy_(lin_state_dict[f'lin{i}.model.1.weight'])
        return self

    def features(self, im):
        if FOLD_SCALING:   # the ScalingLayer folded into the first layer's pass
            return self.net(im, self.shift, self.scale)
        return self.net((im - self.shift) / self.scale)

    def target_features(self, in1):
        """The second input's feature taps without gradient (forward(in0, f1=...) consumes them:
        the inversion computes them for the target on a side stream)."""
        with torch.no_grad():
            return self.features(in1)

    def forward(self, in0, in1=None, f1=None):
        f0 = self.features(in0)
        if f1 is None:
            with torch.no_grad() if not in1.requires_grad else _null():
                f1 = self.features(in1)
        from . import producer_ops
        return sum(producer_ops.lpips_head(a, b, lin.weight.view(-1))
                   for a, b, lin in zip(f0, f1, self.lins))[:, None]


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

