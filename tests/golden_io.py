"""Load the committed golden vectors (tests/golden/*.npz, produced by gen_golden.py)."""

import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
RENDER_CASES = ['p3d', 'shapenet', 'cub', 'persp_center_bbox']
EXTRAS_CASES = ['extras_ns', 'extras_nw', 'extras_coords']   # eval outputs, no gradients


def load(name):
    z = np.load(os.path.join(GOLDEN, f'{name}.npz'))   # allow_pickle stays False
    d = {}
    meta = {}
    for k in z.files:
        if k.startswith('meta_'):
            meta[k[5:]] = z[k].item()
        else:
            d[k] = torch.from_numpy(z[k].copy())
    return d, meta


def field_from(d, meta):
    from oracle.render_oracle import Field
    return Field(planes=d['planes'], w1=d['w1'], b1=d['b1'], w2=d['w2'], b2=d['b2'],
                 palette=d['palette'], alpha=d['alpha'], beta=d['beta'],
                 scene_range=float(meta['scene_range']))
