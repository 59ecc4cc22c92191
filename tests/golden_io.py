"""Load the committed golden vectors (tests/golden/*.npz, produced by gen_golden.py)."""

import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
RENDER_CASES = ['p3d', 'shapenet', 'cub', 'persp_center_bbox', 'inside']
VARIANT_CASES = ['rgbhead', 'nerfdensity', 'nerf_rgbhead', 'attn5']   # attention_values 0 / 5, use_sdf False
VIEWDIR_CASES = ['viewdir', 'viewdir_rgbhead']               # --use_viewdir
ZBUFFER_CASES = ['zbuffer']        # eval_nusc_persp.py's render copy (z-buffer depth)
EXTRAS_CASES = ['extras_ns', 'extras_nw', 'extras_coords']   # eval outputs, no gradients


def load(name):
    z = np.load(os.path.join(GOLDEN, f'{name}.npz'))   # allow_pickle stays False
    d = {}
    meta = {}
    for k in z.files:
        if k.startswith('meta_'):
            meta[k[5:]] = z[k].item()
        elif z[k].dtype.kind == 'U':
            d[k] = z[k]                            # text (state_dict key/shape lists)
        else:
            d[k] = torch.from_numpy(z[k].copy())
    return d, meta


def viewdir_params(d):
    """The fixture's ViewDirectionMapper state_dict (keys 'vd_<name>'), or None."""
    p = {k[3:]: v for k, v in d.items() if k.startswith('vd_')}
    return p or None


def field_from(d, meta):
    from oracle.render_oracle import Field
    return Field(planes=d['planes'], w1=d['w1'], b1=d['b1'], w2=d['w2'], b2=d['b2'],
                 palette=d.get('palette'), alpha=d.get('alpha'), beta=d.get('beta'),
                 scene_range=float(meta['scene_range']),
                 attention_values=int(meta.get('attention_values', 10)),
                 use_sdf=bool(meta.get('use_sdf', 1)), viewdir=viewdir_params(d))


PRODUCER_SKIP = ('resample_filter', 'noise_const')


def seeded_parameters(named_shapes, seed):
    """Deterministic weights for a generator's parameters, shared by gen_golden.py (applied to
    the reference Generator) and the tests (applied to nfi.producer): each tensor drawn by numpy
    from (seed, crc32(name)), so the fixture stores no weights.  Modulation-affine biases sit
    around 1 (their init), other biases around 0, alpha/beta keep the reference's init."""
    import zlib
    out = {}
    for name, shape in named_shapes:
        if name.endswith(PRODUCER_SKIP):
            continue
        if name == 'alpha':
            v = np.ones(shape, np.float32)
        elif name == 'beta':
            v = np.full(shape, 0.1, np.float32)
        else:
            rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
            v = rng.standard_normal(shape, dtype=np.float32)
            if name.endswith('affine.bias'):
                v = 1 + 0.1 * v
            elif name.endswith('bias'):
                v = 0.1 * v
        out[name] = torch.from_numpy(v)
    return out


def load_seeded(module, seed):
    """Overwrite `module`'s parameters with seeded_parameters(...) (buffers untouched)."""
    shapes = [(k, tuple(p.shape)) for k, p in module.named_parameters()]
    vals = seeded_parameters(shapes, seed)
    with torch.no_grad():
        for k, p in module.named_parameters():
            p.copy_(vals[k])
    return module
