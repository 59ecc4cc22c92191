"""The view-direction mapper of the reference's field (--use_viewdir; models/generator.py:189-252).

Its per-ray trunk — ViewDirectionMapper.forward up to `x` (generator.py:223-238): EqualizedLinear
3->64, two residual pairs of (EqualizedLinear 64->64 without bias, LayerNorm, LeakyReLU 0.2) scaled
by sqrt(2)/2, EqualizedLinear 64->64 + LeakyReLU, EqualizedLinear 64->32 — runs here on the
caller's module (the reference's own `Generator.viewdir_mapper`, or any module with the same
sub-module names), once per ray: B*H*W rows of a small MLP.  The per-sample part of its closure
(generator.py:242-250: output(leaky_relu(x + features))) runs inside the HIP render kernels
(NFI_HEAD_VIEWDIR), which also return dL/d x so autograd reaches the ray directions through
this trunk.
"""

from __future__ import annotations

import math

import torch


def viewdir_trunk(mapper, viewdir: torch.Tensor) -> torch.Tensor:
    """generator.py:223-238 on `mapper`'s layers: viewdir [..., 1, 3] -> x [..., 1, 32]."""
    scale = math.sqrt(2) / 2
    relu = mapper.relu
    x = relu(mapper.fc0(viewdir))
    shortcut = x
    x = relu(mapper.norm1(mapper.fc1(x)))
    x = relu(mapper.norm2(mapper.fc2(x)))
    x = (x + shortcut).mul_(scale)
    shortcut = x
    x = relu(mapper.norm3(mapper.fc3(x)))
    x = relu(mapper.norm4(mapper.fc4(x)))
    x = (x + shortcut).mul_(scale)
    x = relu(mapper.fc5(x))
    x = mapper.fc6(x)
    assert x.shape[-2] == 1, x.shape
    return x


class ViewDirectionMapper(torch.nn.Module):
    """The reference module's structure and state_dict keys (generator.py:189-221): a reference
    checkpoint's `viewdir_mapper.*` entries load into it strictly.  Its trunk runs through
    viewdir_trunk; `output` is read by the renderer (ops.pack_viewdir_head)."""

    def __init__(self, output_size: int, num_features: int = 32):
        super().__init__()
        from .producer import EqualizedLinear
        h = 64
        self.hidden_size = h
        self.fc0 = EqualizedLinear(3, h)
        for i in range(1, 5):
            setattr(self, f'fc{i}', EqualizedLinear(h, h, bias=False))
            setattr(self, f'norm{i}', torch.nn.LayerNorm(h, elementwise_affine=True))
        self.fc5 = EqualizedLinear(h, h)
        self.fc6 = EqualizedLinear(h, num_features)
        self.output = EqualizedLinear(num_features, output_size)
        with torch.no_grad():
            self.output.weight.zero_()
            self.output.bias.zero_()
        self.relu = torch.nn.LeakyReLU(0.2)

    def forward(self, viewdir):
        return viewdir_trunk(self, viewdir)
