"""Probe of the inversion step's convolution-heavy callers on one GPU: LPIPS-VGG fwd+bwd over
the 16 x B augmented copies and the producer fwd+bwd, with MIOpen's default heuristic solution vs
find mode (torch.backends.cudnn.benchmark) and NCHW vs channels_last.
Usage (GPU box): python scripts/conv_probe.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import lpips, producer  # noqa: E402


def timeit(fn, reps=5):
    fn()
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def lpips_case(B, cl, dev):
    net = lpips.LPIPS().to(dev)
    n = 16 * B
    x = torch.tanh(torch.randn(n, 3, 128, 128, device=dev))
    y = torch.tanh(torch.randn(n, 3, 128, 128, device=dev))
    if cl:
        net = net.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
        y = y.contiguous(memory_format=torch.channels_last)
    x.requires_grad_()

    def step():
        x.grad = None
        net(x, y).sum().backward()
    return timeit(step)


def producer_case(B, cl, dev):
    torch.manual_seed(0)
    gen = producer.InversionGenerator(scene_range=1.4).to(dev).requires_grad_(False)
    if cl:
        gen = gen.to(memory_format=torch.channels_last)
    ws = torch.randn(B, 15, 512, device=dev, requires_grad=True)

    def step():
        ws.grad = None
        planes, pal = gen.planes_and_palette(ws)
        (planes.float().square().mean() + pal.sum()).backward()
    return timeit(step)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda:0')
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for cl in (False, True):
            print(f'B={B} cudnn.benchmark={bench} channels_last={cl}: LPIPS fwd+bwd '
                  f'{lpips_case(B, cl, dev):.2f} ms  producer fwd+bwd {producer_case(B, cl, dev):.2f} ms',
                  flush=True)


if __name__ == '__main__':
    main()
