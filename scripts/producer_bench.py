"""Time the producer (synthesis + palette mapper) fwd+bwd to the latent on one GPU, per layer kind.
Usage (GPU box): python scripts/producer_bench.py [B] [--channels-last] [--torch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import producer  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8
    cl = '--channels-last' in sys.argv
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    backend = 'torch' if '--torch' in sys.argv else 'hip'   # --torch: the oracle's reference op sequence
    gen = producer.InversionGenerator(1.4).to(dev).requires_grad_(False)
    if backend == 'torch':
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
        from oracle.producer_oracle import ReferenceProducer
        gen = ReferenceProducer(gen)
    if cl:
        gen = gen.to(memory_format=torch.channels_last)
    ws = torch.randn(B, 15, 512, device=dev, requires_grad=True)
    g = torch.randn(B, 3, 32, 256, 256, device=dev)

    def step():
        planes, pal = gen.planes_and_palette(ws)
        ((planes * g).sum() + pal.sum()).backward()
        ws.grad = None

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    with torch.no_grad():
        t0 = time.perf_counter()
        for _ in range(n):
            gen.planes_and_palette(ws)
        torch.cuda.synchronize()
        dtf = (time.perf_counter() - t0) / n
    print(f'B={B} backend={backend} channels_last={cl}: fwd+bwd {dt * 1e3:.2f} ms  fwd {dtf * 1e3:.2f} ms  '
          f'({dt / B * 1e3:.2f} ms/image)')


if __name__ == '__main__':
    main()
