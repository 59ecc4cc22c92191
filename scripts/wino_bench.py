"""LPIPS-VGG trunk on one GPU with MIOpen vs the Winograd F(4,3) path (nfi.conv): the prediction
pass (fwd+bwd over 16 x B copies) and the target pass (forward, no grad).
Usage (GPU box): python scripts/wino_bench.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import lpips  # noqa: E402


def timeit(fn, reps=10):
    fn()
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    net = lpips.LPIPS().to(dev)
    n = 16 * B
    x = torch.tanh(torch.randn(n, 3, 128, 128, device=dev)).requires_grad_()
    y = torch.tanh(torch.randn(n, 3, 128, 128, device=dev))
    res = {}
    for wino in (False, True):
        lpips.VGG16Features.winograd = wino
        f1 = net.target_features(y)

        def pred():
            x.grad = None
            net(x, f1=f1).sum().backward()

        res[wino] = (timeit(pred), timeit(lambda: net.target_features(y)))
        print(f'B={B} winograd={wino}: prediction fwd+bwd {res[wino][0]:.2f} ms, '
              f'target fwd {res[wino][1]:.2f} ms', flush=True)


if __name__ == '__main__':
    main()
