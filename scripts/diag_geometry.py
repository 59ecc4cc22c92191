"""Bitwise comparison of the HIP ray geometry (ro, rd, near, far, coarse depths) with the oracle."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'nerf-from-image_amd'), ROOT]
import torch
from gpu_helpers import run_hip, run_oracle, synthetic_inputs

for kw in [dict(scene_range=1.4, seed=3), dict(scene_range=0.55, seed=11, flipped=False, randomize=False),
           dict(scene_range=2.0, seed=8, ortho=True)]:
    inp, meta = synthetic_inputs(B=2, H=8, W=8, S=64, R=32, **kw)
    dbg = {}
    run_hip(inp, meta, torch.device('cuda:0'), debug=dbg, with_grad=False)
    ref = run_oracle(inp, meta, with_grad=False, return_intermediates=True)['inter']
    for k in ['ro', 'rd', 'near', 'far', 'z_coarse']:
        a = dbg[k].cpu().reshape(-1)
        b = ref[k].reshape(-1)
        ne = (a != b)
        print(kw, k, 'mismatch', int(ne.sum()), '/', a.numel(), 'maxdiff', float((a - b).abs().max()))
        if ne.any() and k in ('rd', 'ro'):
            i = int(ne.nonzero()[0])
            print('   first', i, a[i].item(), b[i].item())
