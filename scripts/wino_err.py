"""Where does the Winograd LPIPS image-gradient error come from?  fp64 truth vs hip backend with
the Winograd forward only / data gradient only / both.  Usage (GPU box)."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import conv, lpips  # noqa: E402


def ev(net, a, b):
    a = a.detach().clone().requires_grad_()
    out = net(a, b)
    out.sum().backward()
    return out.detach().double().cpu(), a.grad.double().cpu()


DEV = torch.device('cuda:0')
torch.manual_seed(0)
from oracle.producer_oracle import ReferenceLPIPS   # noqa: E402
net = lpips.LPIPS().to(DEV)
a = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV))
b = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV))
ref, gref = ev(ReferenceLPIPS(copy.deepcopy(net).double().cpu()), a.double().cpu(), b.double().cpu())
print('grad max/rms', float(gref.abs().max() / gref.square().mean().sqrt()))
for fw, dg in ((False, False), (True, False), (False, True), (True, True)):
    lpips.VGG16Features.winograd = True
    conv.ENABLED = True
    conv.DGRAD = dg
    if not fw and not dg:
        conv.ENABLED = False
    if not fw and dg:
        print('(dgrad-only needs the forward on winograd: skipped)')
        continue
    o, g = ev(net, a, b)
    e = (g - gref)
    print(f'winograd fwd={fw} dgrad={dg}: loss {float((o - ref).abs().max() / ref.abs().max()):.2e} '
          f'grad relL2 {float(e.norm() / gref.norm()):.2e} max/max {float(e.abs().max() / gref.abs().max()):.2e}')
