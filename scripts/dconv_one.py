"""One direct-convolution layer (nfi_dconv3x3) launched REPS times, for rocprofv3 counter passes on the
kernel alone.  Usage: python scripts/dconv_one.py [N Ci Co H [reps [mask]]]  (default: 64 64 64 128,
the LPIPS conv1_2 layer)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd')]
import torch  # noqa: E402

from nfi import conv  # noqa: E402

DEV = torch.device('cuda:0')


def main():
    a = [int(v) for v in sys.argv[1:]]
    N, Ci, Co, H = a[:4] if len(a) >= 4 else (64, 64, 64, 128)
    reps = a[4] if len(a) > 4 else 20
    mask = len(a) > 5 and a[5] == 1
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.relu(torch.randn((N, Ci, H, H), device=DEV, generator=g))
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    yv = torch.randn((N, Ci, H, H), device=DEV, generator=g) if mask else None
    U, _ = conv.weights(w)
    assert conv._direct_ok(U, x)   # (packs the direct weight)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 2):
        if i == 2:
            e0.record()
        if mask:
            conv._direct(x, U, relu_y=yv)
        else:
            conv._direct(x, U, b, True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f'{N}x{Ci}->{Co} @{H}^2: {ms:.3f} ms per call (absmax + conv), {2.0 * N * Co * Ci * 9 * H * H / ms / 1e9:.0f} TF')


if __name__ == '__main__':
    main()
