"""Which part of the inversion step survives HIP-graph capture?  Captures one piece per process:
  render    rays + fused render fwd+bwd of a synthetic field (nfi HIP kernels only)
  producer  synthesis network + AttentionMapper fwd+bwd (MIOpen, hipBLASLt, Winograd, epilogues)
  adam      a capturable Adam step on a few tensors
  lpips     LPIPS-VGG fwd+bwd (Winograd, MIOpen first layer, distance head)
  step      the whole L1 inversion step
Usage (GPU box): python scripts/graph_probe.py <piece>; exits 0 after capture + 3 replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

import nfi  # noqa: E402
from nfi import inversion, lpips, ops, producer  # noqa: E402
from nfi.synthetic import inversion_batch  # noqa: E402

DEV = torch.device('cuda:0')


def capture(fn, warm=2):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    print('capturing', flush=True)
    with torch.cuda.graph(g):
        out = fn()
    print('captured', flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print('replayed', flush=True)
    return out


def main():
    piece = sys.argv[1]
    torch.manual_seed(0)
    if piece == 'render':
        b = inversion_batch(2, 64, 64, 32, 64, 1.4, 0, flipped=True, device=DEV)
        f = b['field']
        cam = b['cam'].detach().requires_grad_()

        def fn():
            f.planes.grad = f.palette.grad = cam.grad = None
            rgb = nfi.render(f, 64, 64, cam, b['focal'], None, None, None, 32)[0]
            rgb.square().sum().backward()
            return rgb
        capture(fn)
    elif piece == 'producer':
        gen = producer.InversionGenerator(1.4).to(DEV).requires_grad_(False)
        ws = torch.randn(2, 15, 512, device=DEV, requires_grad=True)

        def fn():
            ws.grad = None
            planes, pal = gen.planes_and_palette(ws)
            (planes.square().mean() + pal.sum()).backward()
            return planes
        capture(fn)
    elif piece == 'adam':
        p = torch.randn(4, 16, device=DEV, requires_grad=True)
        opt = torch.optim.Adam([p], lr=1e-3, capturable=True)

        def fn():
            opt.zero_grad(set_to_none=True)
            p.square().sum().backward()
            opt.step()
        capture(fn)
    elif piece == 'lpips':
        net = lpips.LPIPS().to(DEV)
        x = torch.tanh(torch.randn(4, 3, 64, 64, device=DEV)).requires_grad_()
        y = torch.tanh(torch.randn(4, 3, 64, 64, device=DEV))

        def fn():
            x.grad = None
            out = net(x, y)
            out.sum().backward()
            return out
        capture(fn)
    elif piece == 'step':
        sys.path.insert(0, os.path.join(ROOT, 'tests'))
        from test_producer import inversion_setup
        gen, d, meta, cfg = inversion_setup(DEV)
        nfi.configure(scene_range=float(meta['scene_range']), white_background=False)
        cfg.steps, cfg.resolution, cfg.samples = 5, 64, 32
        target = torch.nn.functional.interpolate(d['target'].permute(0, 3, 1, 2), size=(64, 64),
                                                 mode='bilinear', align_corners=False).permute(0, 2, 3, 1)
        res = inversion.invert(gen, target.contiguous(), d['cam0'], d['focal0'], d['w_init'], cfg)
        print(res.losses)
    ops.KERNEL_TIMERS = None
    print(f'{piece}: ok', flush=True)


if __name__ == '__main__':
    main()
