"""The tri-plane producer of the inversion step, caller side: the parts of the
reference Generator that turn a latent ws [b,15,512] into the renderer's inputs —
StyleGAN2 synthesis network -> tri-planes [b,3,32,256,256] (stylegan.py:293-490,
generator.py:475-477), AttentionMapper -> palette [b,10,3] (generator.py:132-186,
455-462) — plus the mapping network used for the average latent (stylegan.py:228-290,
generator.py:263-282) and the frozen SDF decoder weights.

One implementation, on the device: the convolutions' products are hipBLASLt GEMMs (3x3:
Winograd F(4,3), nfi/conv.py; stride-2 up-sampling: one GEMM over the 9 taps + HIP tap scatter
fused with the FIR and epilogue; 1x1 to-planes: one batched GEMM with the modulation folded into a
per-image weight) and everything between them runs in the fused HIP kernels of
csrc/nfi_producer.hip (producer_ops.py): modulation backward, demodulation + bias + gain +
leaky-ReLU epilogue, the skip-image upsample + add; the styles and demodulation coefficients of
all layers as two batched products (style_bank).  Device tensors only (CPU tensors raise).  The
reference's op sequence in plain PyTorch over these modules' parameters is test infrastructure:
oracle/producer_oracle.py (the tests' CPU loop and bench.py's cpu_baseline).
Parameter and buffer names equal the reference Generator's state_dict keys, so a G_ema
checkpoint loads with `load_state_dict(sd)`.  Pinned by tests/golden/producer.npz
(tests/test_gpu_inversion.py; the oracle restatement by tests/test_producer.py on CPU).  The HIP renderer
consumes it through `nfi.render(generator, ...)` exactly as it consumes the reference Generator.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

SQRT2 = math.sqrt(2.0)
def _hip():
    from . import producer_ops
    return producer_ops


def _conv():
    from . import conv
    return conv


def blur_kernel() -> torch.Tensor:
    """[1,3,3,1] x [1,3,3,1] / 64 (stylegan.py `bilinear_filter`)."""
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = k[:, None] * k[None, :]
    return k / k.sum()


def frozen_value(mod: nn.Module, key: str, fn, *params):
    """fn() cached on `mod` while `params` are frozen and unmodified: the gain-scaled weights and
    the demodulation sums of squares are functions of the generator's parameters only, which the
    inversion does not train (run.py:630-632), so they are computed once instead of every step.
    Invalidated by any in-place update of a parameter (tensor version counter) or a new tensor;
    a parameter that requires grad is never cached."""
    tag = tuple((None if p is None else (p.data_ptr(), p._version, p.requires_grad, p.device))
                for p in params)
    if any(p is not None and p.requires_grad for p in params) and torch.is_grad_enabled():
        return fn()
    cache = mod.__dict__.setdefault('_frozen_cache', {})
    hit = cache.get(key)
    if hit is None or hit[0] != tag:
        with torch.no_grad():
            hit = (tag, fn())
        cache[key] = hit
    return hit[1]


class EqualizedLinear(nn.Module):
    """y = x (W * lr/sqrt(in))^T + b * lr (stylegan.py:148-180)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, activate: bool = False,
                 lr_multiplier: float = 1.0, bias_init: float = 0.0):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(out_features, in_features) / lr_multiplier)
        self.bias = nn.Parameter(torch.full((out_features,), float(bias_init))) if bias else None
        self.weight_gain = lr_multiplier / math.sqrt(in_features)
        self.bias_gain = lr_multiplier
        self.activate = activate

    def forward(self, x):
        w, b = frozen_value(self, 'scaled', lambda: (
            self.weight * self.weight_gain, None if self.bias is None else self.bias * self.bias_gain),
            self.weight, self.bias)
        y = F.linear(x, w, b)
        if self.activate:
            y = F.leaky_relu(y * SQRT2, 0.2)
        return y


class ModulatedConv(nn.Module):
    """SynthesisLayer (stylegan.py:293-360): style-modulated 3x3 conv with demodulation, optional
    2x upsampling (transposed conv + FIR), bias, sqrt(2) gain, leaky ReLU.  The modulation scales
    the input channels and demodulation the output channels, so the convolution itself uses the
    shared weight (one conv for the whole batch)."""

    def __init__(self, in_ch: int, out_ch: int, w_dim: int, resolution: int, up: bool = False):
        super().__init__()
        self.up = up
        self.affine = EqualizedLinear(w_dim, in_ch, bias_init=1.0)
        self.weight = nn.Parameter(torch.randn(out_ch, in_ch, 3, 3))
        self.bias = nn.Parameter(torch.zeros(out_ch))
        # noise inputs (disabled in the inversion generator: disable_stylegan_noise=True)
        self.noise_strength = nn.Parameter(torch.zeros([]))
        self.register_buffer('noise_const', torch.randn(resolution, resolution))
        self.register_buffer('resample_filter', blur_kernel())

    def forward(self, x, w, pre=None):
        ops = _hip()
        if pre is None:
            styles = self.affine(w)
            w2 = frozen_value(self, 'w2', lambda: self.weight.square().sum(dim=(2, 3)), self.weight)  # [out, in]
            dcoefs = (styles.square() @ w2.t() + 1e-8).rsqrt()                # [b, out]
        else:                                  # from SynthesisNetwork's style bank
            styles, dcoefs = pre
        if self.up:
            return ops.up_conv_act(ops.scale(x, styles), self.weight, dcoefs, self.bias, SQRT2)
        return ops.act(_conv().modulated_conv3x3(x, styles, self.weight), dcoefs, self.bias, SQRT2)


class ToPlanes(nn.Module):
    """OutputLayer (stylegan.py:363-384): modulated 1x1 conv without demodulation, plus bias."""

    def __init__(self, in_ch: int, out_ch: int, w_dim: int):
        super().__init__()
        self.affine = EqualizedLinear(w_dim, in_ch, bias_init=1.0)
        self.weight = nn.Parameter(torch.randn(out_ch, in_ch, 1, 1))
        self.bias = nn.Parameter(torch.zeros(out_ch))
        self.weight_gain = 1.0 / math.sqrt(in_ch)

    out_layout = 'nhwc'     # the last resolution's layer is set to 'planes'

    def forward(self, x, w, pre=None):
        styles = self.affine(w) * self.weight_gain if pre is None else pre
        # channels-last (the skip-image chain's layout: its last image is the renderer's
        # texel-major planes, no conversion pass); bias added in up_add
        return _hip().modulated_conv1x1(x, styles, self.weight, layout=self.out_layout)


class SynthesisBlock(nn.Module):
    """One resolution of the synthesis network (stylegan.py:387-446)."""

    def __init__(self, in_ch: int, out_ch: int, w_dim: int, resolution: int, img_ch: int):
        super().__init__()
        self.in_ch = in_ch
        if in_ch == 0:
            self.const = nn.Parameter(torch.randn(out_ch, resolution, resolution))
        else:
            self.conv0 = ModulatedConv(in_ch, out_ch, w_dim, resolution, up=True)
        self.conv1 = ModulatedConv(out_ch, out_ch, w_dim, resolution)
        self.torgb = ToPlanes(out_ch, img_ch, w_dim)
        self.register_buffer('resample_filter', blur_kernel())
        self.num_conv = 1 if in_ch == 0 else 2

    def forward(self, x, img, ws, bank=None):
        """ws: this block's rows of the latent; bank: their precomputed (styles, dcoefs) per layer
        in the order conv0, conv1, torgb (SynthesisNetwork.style_bank), or None."""
        k = 0
        pre = bank or (None, None, None)
        if self.in_ch == 0:
            x = self.const[None].expand(ws[0].shape[0], -1, -1, -1)
        else:
            x = self.conv0(x, ws[k], pre[0])
            k += 1
        x = self.conv1(x, ws[k], pre[k])
        y = self.torgb(x, ws[k + 1], pre[k + 1])
        return x, _hip().up_add(img, y, self.torgb.bias)


class SynthesisNetwork(nn.Module):
    """ws [b, num_ws, w_dim] -> image [b, img_ch, res, res] (stylegan.py:449-490); blocks at
    4, 8, ..., res with min(channel_base/r, channel_max) channels."""

    def __init__(self, w_dim: int = 512, img_resolution: int = 256, img_channels: int = 96,
                 channel_base: int = 32768, channel_max: int = 512):
        super().__init__()
        self.resolutions = [2 ** i for i in range(2, int(math.log2(img_resolution)) + 1)]
        ch = {r: min(channel_base // r, channel_max) for r in self.resolutions}
        self.num_ws = 0
        for r in self.resolutions:
            blk = SynthesisBlock(ch[r // 2] if r > 4 else 0, ch[r], w_dim, r, img_channels)
            setattr(self, f'b{r}', blk)
            self.num_ws += blk.num_conv
        self.num_ws += 1   # the last block's toRGB
        # the last image is the tri-planes: written texel-major ([b, 3, 32, R, R] in the renderer's
        # [b, 3, R, R, 32] storage), so render() reads it with no conversion pass
        getattr(self, f'b{self.resolutions[-1]}').torgb.out_layout = 'planes'

    def forward(self, ws, noise_mode: str = 'const'):
        # ws [b, num_ws, w_dim] or its rows (a sequence of [b, w_dim]); the rows are split once
        # (one unbind: its backward is one stack, not a zero-filled [b, num_ws, w_dim] gradient and
        # an accumulation per slice)
        bank = None
        if torch.is_tensor(ws) and ws.is_cuda:
            bank = iter(self.style_bank(ws))
        rows = ws.unbind(1) if torch.is_tensor(ws) else ws
        x = img = None
        k = 0
        for r in self.resolutions:
            blk = getattr(self, f'b{r}')
            pre = None if bank is None else [next(bank) for _ in range(blk.num_conv + 1)]
            x, img = blk(x, img, rows[k:k + blk.num_conv + 1], pre)
            k += blk.num_conv
        return img

    def _bank_layers(self):
        """(module, latent row, is_conv) of every modulated layer in execution order."""
        out, base = [], 0
        for r in self.resolutions:
            blk = getattr(self, f'b{r}')
            k = base                      # SynthesisNetwork.forward hands block r rows[base:]
            if blk.in_ch:
                out.append((blk.conv0, k, True))
                k += 1
            out.append((blk.conv1, k, True))
            out.append((blk.torgb, k + 1, False))
            base += blk.num_conv
        return out

    def style_bank(self, ws):
        """The styles (affine of the layer's latent row, stylegan.py:337 / :375-377) and the
        demodulation coefficients (:140-142) of all 21 modulated layers as two batched products
        instead of ~35 small GEMMs and their elementwise tails: S = X W^T + b over the stacked
        gain-folded affine weights ([21, 512, 512], zero-padded rows), D = rsqrt(S^2 W2^T + 1e-8)
        over the stacked sums of squared conv weights ([14, 512, 512]).  Frozen parameters only
        (the stacks are built once per parameter version, frozen_value).  Returns, per layer in
        execution order, (styles [b, in], dcoefs [b, out]) for convolutions and styles for toRGB
        (its 1/sqrt(in) weight gain folded in)."""
        layers = self._bank_layers()
        params = []
        for m, _, conv in layers:
            params += [m.affine.weight, m.affine.bias] + ([m.weight] if conv else [])

        def build():
            dev = ws.device
            L = len(layers)
            wdim = layers[0][0].affine.weight.shape[1]
            cmax = max(m.affine.weight.shape[0] for m, _, _ in layers)
            conv_ids = [i for i, (_, _, c) in enumerate(layers) if c]
            omax = max(layers[i][0].weight.shape[0] for i in conv_ids)
            A = torch.zeros((L, cmax, wdim), device=dev)
            bias = torch.zeros((L, 1, cmax), device=dev)
            W2 = torch.zeros((len(conv_ids), omax, cmax), device=dev)
            for i, (m, _, conv) in enumerate(layers):
                g = 1.0 if conv else m.weight_gain
                n = m.affine.weight.shape[0]
                A[i, :n] = m.affine.weight * (m.affine.weight_gain * g)
                bias[i, 0, :n] = m.affine.bias * (m.affine.bias_gain * g)
            for j, i in enumerate(conv_ids):
                w = layers[i][0].weight
                W2[j, :w.shape[0], :w.shape[1]] = w.square().sum(dim=(2, 3))
            rows = torch.tensor([k for _, k, _ in layers], device=dev)
            return A.transpose(1, 2), bias, W2.transpose(1, 2), rows, torch.tensor(conv_ids, device=dev)

        At, bias, W2t, rows, conv_ids = frozen_value(self, 'style_bank', build, *params)
        S = torch.baddbmm(bias, ws.index_select(1, rows).transpose(0, 1), At)        # [L, b, cmax]
        D = (torch.bmm(S.index_select(0, conv_ids).square(), W2t) + 1e-8).rsqrt()   # [Lc, b, omax]
        b = ws.shape[0]
        s_w = [m.affine.weight.shape[0] for m, _, _ in layers]
        d_w = [m.weight.shape[0] for m, _, c in layers if c]
        styles = _PackRows.apply(S, _pack_index(self, 'styles', S.shape, s_w, S.device), b, s_w)
        dcoefs = iter(_PackRows.apply(D, _pack_index(self, 'dcoefs', D.shape, d_w, D.device), b, d_w))
        return [(s, next(dcoefs)) if conv else s for (m, _, conv), s in zip(layers, styles)]


def _pack_index(mod, key, shape, widths, dev):
    """Flat positions in a padded [L, b, W] stack of each layer's [b, n_l] block, in layer order
    (built once per shape on the device: no host copy inside a step)."""
    cache = mod.__dict__.setdefault('_pack_cache', {})
    k = (key, tuple(shape), tuple(widths), dev)
    idx = cache.get(k)
    if idx is None:
        L, b, W = shape
        idx = torch.cat([(l * b * W + torch.arange(b)[:, None] * W + torch.arange(n)[None, :]).reshape(-1)
                         for l, n in enumerate(widths)]).to(dev)
        cache[k] = idx
    return idx


class _PackRows(torch.autograd.Function):
    """A padded [L, b, W] stack -> its L blocks [b, n_l] as contiguous tensors (views of one packed
    buffer): one gather forward; backward one concatenation of the gradients and one index_copy
    into the zero-padded stack (instead of a copy per sliced layer forward and a zero-fill + copy
    per layer backward)."""

    @staticmethod
    def forward(ctx, X, idx, b, widths):
        flat = X.reshape(-1).index_select(0, idx)
        ctx.save_for_backward(idx)
        ctx.shape, ctx.b, ctx.widths = X.shape, b, widths
        return tuple(t.view(b, n) for t, n in zip(flat.split([b * n for n in widths]), widths))

    @staticmethod
    def backward(ctx, *grads):
        idx, = ctx.saved_tensors
        b = ctx.b
        flat = torch.cat([(g if g is not None else idx.new_zeros((b, n), dtype=torch.float32)).reshape(-1)
                          for g, n in zip(grads, ctx.widths)])
        G = flat.new_zeros(ctx.shape).view(-1)
        G.index_copy_(0, idx, flat)
        return G.view(ctx.shape), None, None, None


class MappingNetwork(nn.Module):
    """z -> w (stylegan.py:228-290) with normalize_latent, 2 layers, lr multiplier 0.01."""

    def __init__(self, z_dim: int = 512, w_dim: int = 512, num_ws: int = 15, num_layers: int = 2,
                 lr_multiplier: float = 0.01):
        super().__init__()
        self.z_dim, self.w_dim, self.num_ws, self.num_layers = z_dim, w_dim, num_ws, num_layers
        dims = [z_dim] + [w_dim] * num_layers
        for i in range(num_layers):
            setattr(self, f'fc{i}', EqualizedLinear(dims[i], dims[i + 1], activate=True,
                                                    lr_multiplier=lr_multiplier))

    def forward(self, z, c=None):
        x = z * (z.square().mean(dim=1, keepdim=True) + 1e-8).rsqrt()
        for i in range(self.num_layers):
            x = getattr(self, f'fc{i}')(x)
        return x.unsqueeze(1).repeat(1, self.num_ws, 1)


class MappingWrapper(nn.Module):
    def __init__(self, backbone: MappingNetwork):
        super().__init__()
        self.backbone = backbone

    def forward(self, z, c=None):
        return self.backbone(z, c)

    @torch.no_grad()
    def get_average_w(self, n_samples: int = 10000, generator=None):
        """Mean w over n_samples z ~ N(0, I) (generator.py:263-271)."""
        dev = self.backbone.fc0.weight.device
        z = torch.randn((n_samples, self.backbone.z_dim), generator=generator).to(dev)
        return self(z).mean(dim=0, keepdim=True)


class ConditionalLayerNorm(nn.Module):
    """LayerNorm (no affine) with (1 + gamma(z)) scale and beta(z) shift (generator.py:42-60): its
    parameters; PaletteMapper applies all four norms from one batched projection (_conditions)."""

    def __init__(self, ch: int, emb_dim: int):
        super().__init__()
        self.ch = ch
        self.fc_gamma = EqualizedLinear(emb_dim, ch)
        self.fc_beta = EqualizedLinear(emb_dim, ch)


def wide_sigmoid_rescaled(x):
    """MipNeRF wide sigmoid rescaled to [-1.002, 1.002] (generator.py:37-39)."""
    return torch.sigmoid(x) * 2.004 - 1.002


class PaletteMapper(nn.Module):
    """AttentionMapper (generator.py:132-186): w_tex -> 10 RGB attention values."""

    def __init__(self, latent_dim: int = 512, num_values: int = 10, hidden: int = 512):
        super().__init__()
        self.num_values = num_values
        self.const = nn.Parameter(torch.randn(1, hidden))
        for i in range(1, 5):
            setattr(self, f'fc{i}', EqualizedLinear(hidden, hidden, bias=False))
            setattr(self, f'norm{i}', ConditionalLayerNorm(hidden, latent_dim))
        self.fc5 = EqualizedLinear(hidden, hidden)
        self.fc_values = EqualizedLinear(hidden, num_values * 3)

    def forward(self, c):
        scale = SQRT2 / 2
        x = self.const.expand(c.shape[0], -1)
        cond = self._conditions(c)
        for pair in ((1, 2), (3, 4)):
            shortcut = x
            for i in pair:
                h = getattr(self, f'fc{i}')(x)
                # (1 + gamma_i(c)) and beta_i(c) from the one batched projection
                g1, b = cond[2 * (i - 1)], cond[2 * (i - 1) + 1]
                if h.is_cuda and h.shape[-1] <= 1024:
                    x = _hip().cond_norm_act(h, g1, b)        # one HIP kernel each way
                else:
                    x = F.leaky_relu(torch.addcmul(b, g1, F.layer_norm(h, (h.shape[-1],))), 0.2)
            x = (x + shortcut) * scale
        x = F.leaky_relu(self.fc5(x), 0.2)
        return wide_sigmoid_rescaled(self.fc_values(x).view(-1, self.num_values, 3))

    def _conditions(self, c):
        """The 4 conditional norms' (1 + gamma_i(c), beta_i(c)) (generator.py:42-60) as ONE
        [b,512] x [512, 8*512] product over the stacked gain-scaled weights (the +1 folded into
        gamma's bias), split into 8 views: 1 GEMM and one concatenated gradient instead of 8 GEMMs,
        4 adds and 8 accumulated gradients (frozen weights: built once per parameter version)."""
        norms = [getattr(self, f'norm{i}') for i in range(1, 5)]
        params = []
        for n in norms:
            params += [n.fc_gamma.weight, n.fc_gamma.bias, n.fc_beta.weight, n.fc_beta.bias]

        def build():
            ws, bs = [], []
            for n in norms:
                for lin, one in ((n.fc_gamma, 1.0), (n.fc_beta, 0.0)):
                    ws.append(lin.weight * lin.weight_gain)
                    bs.append(lin.bias * lin.bias_gain + one)
            return torch.cat(ws, 0), torch.cat(bs, 0)

        W, b = frozen_value(self, 'conditions', build, *params)
        return F.linear(c, W, b).split(norms[0].ch, dim=1)


class Decoder(nn.Module):
    """TriplanarDecoder.net weights (generator.py:288-299); evaluated by the HIP renderer."""

    def __init__(self, num_in: int = 32, num_out: int = 10, hidden: int = 64):
        super().__init__()
        self.net = nn.Sequential(EqualizedLinear(num_in, hidden), nn.Softplus(),
                                 EqualizedLinear(hidden, 1 + num_out))


class InversionGenerator(nn.Module):
    """The inversion configuration of the reference Generator (generator.py:334-405:
    latent 512, attention_values=10, use_sdf, no viewdir / encoder / classes, StyleGAN noise
    disabled).  `nfi.render(gen, ...)` renders it; `planes_and_palette(ws)` exposes the producer."""

    def __init__(self, scene_range: float, img_resolution: int = 256):
        super().__init__()
        self.scene_range = scene_range
        self.attention_values = 10
        self.use_sdf = True
        self.use_viewdir = False
        self.use_encoder = False
        self.num_classes = None
        self.mapping_network = MappingWrapper(MappingNetwork(num_ws=15))
        self.synthesis_network = SynthesisNetwork(512, img_resolution, 96)
        self.decoder = Decoder(32, 10)
        self.texture_mapper = PaletteMapper(512, 10)
        self.beta = nn.Parameter(torch.tensor([0.1]))
        self.alpha = nn.Parameter(torch.tensor([1.0]))

    def planes_and_palette(self, ws):
        w_syn, w_tex = ws.split([14, ws.shape[1] - 14], dim=1)    # one split (its backward is one cat)
        palette = self.texture_mapper(w_tex[:, 0])
        planes = self.synthesis_network(w_syn)
        return planes.view(ws.shape[0], 3, 32, planes.shape[-2], planes.shape[-1]), palette
