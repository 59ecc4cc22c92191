"""Run-to-run determinism of d palette (exact) and d planes (float-atomic order) at full size (p3d, B=2); usage: python scripts/determinism_probe.py [S]."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd'), os.path.join(ROOT, 'tests')]
import torch
import nfi
from gpu_helpers import synthetic_inputs

dev = torch.device('cuda:0')
S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
inp, meta = synthetic_inputs(B=2, H=128, W=128, S=S, R=256, scene_range=1.4, seed=0)
nfi.configure(scene_range=1.4)
g = torch.Generator().manual_seed(3)
g_rgb = torch.randn(2, 128, 128, 3, generator=g).to(dev)


def run():
    planes = inp['planes'].to(dev).requires_grad_()
    pal = inp['palette'].to(dev).requires_grad_()
    f = nfi.TriplaneField(planes=planes, palette=pal, w1=inp['w1'].to(dev), b1=inp['b1'].to(dev),
                          w2=inp['w2'].to(dev), b2=inp['b2'].to(dev), alpha=1.0, beta=0.1)
    rgb = nfi.render(f, 128, 128, inp['cam'].to(dev), inp['focal'].to(dev), None, None, None, S, randomize=True,
                     seed=1)[0]
    (rgb * g_rgb).sum().backward()
    torch.cuda.synchronize()
    return pal.grad.clone(), planes.grad.clone()


ref_p, ref_d = run()
for i in range(4):
    p, dpl = run()
    print(i, 'd_palette equal', torch.equal(p, ref_p), float((p - ref_p).abs().max()),
          'd_planes rel', float((dpl - ref_d).norm() / ref_d.norm()))
