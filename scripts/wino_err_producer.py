"""Producer (synthesis 256^2 x 96 + AttentionMapper) d ws against an fp64 truth (torch backend,
float64 on the GPU): torch fp32, hip with MIOpen convolutions, hip with Winograd.  Usage (GPU box)."""
import copy
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import conv, producer  # noqa: E402

DEV = torch.device('cuda:0')
torch.manual_seed(3)
gen = producer.InversionGenerator(1.4).to(DEV).requires_grad_(False)
ws = 0.6 * torch.randn(2, 15, 512, device=DEV)
g = torch.randn(2, 3, 32, 256, 256, device=DEV)


def ev(gn, dtype, be):
    gn.set_backend(be)
    w = ws.to(dtype).detach().clone().requires_grad_()
    planes, pal = gn.planes_and_palette(w)
    ((planes * g.to(dtype)).sum() + pal.sum()).backward()
    return planes.detach().double(), w.grad.double()


t0 = time.time()
g64 = copy.deepcopy(gen).double()
ref = ev(g64, torch.float64, 'torch')
print(f'fp64 truth in {time.time() - t0:.1f} s', flush=True)
for name, be, wino in (('torch fp32', 'torch', True), ('hip miopen', 'hip', False), ('hip winograd', 'hip', True)):
    conv.ENABLED = wino
    p, d = ev(gen, torch.float32, be)
    print(f'{name}: planes max/max {float((p - ref[0]).abs().max() / ref[0].abs().max()):.2e}  '
          f'd ws relL2 {float((d - ref[1]).norm() / ref[1].norm()):.2e}', flush=True)
