"""Split-f16 GEMM (nfi_gemm_split16) vs torch.bmm (hipBLASLt fp32) on the Winograd products of the
inversion step (36 batched [Co x Ci] x [Ci x P]): ms and TFLOP/s (fp32-equivalent, 2 M N K per
product) per shape.  GPU box: python scripts/gemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd'), os.path.join(ROOT, 'tests')]
import torch  # noqa: E402

from test_gpu_gemm import split_gemm  # noqa: E402

DEV = torch.device('cuda:0')
# (Co, Ci, P): LPIPS VGG16 trunk at 128^2 over 4 images x 16 copies (P = 64 (H/4)^2), producer 3x3
# layers at B = 4 (P = 4 (H/4)^2)
SHAPES = [(128, 128, 16384), (256, 128, 4096), (256, 256, 4096), (512, 256, 1024), (512, 512, 1024),
          (512, 512, 256), (256, 256, 16384), (128, 128, 65536), (512, 512, 4096)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    for Co, Ci, P in SHAPES:
        A = torch.randn((36, Co, Ci), device=DEV)
        B = torch.randn((36, Ci, P), device=DEV)
        fl = 2 * 36 * Co * Ci * P
        t_bmm = timeit(lambda: torch.bmm(A, B))
        t_split = timeit(lambda: split_gemm(A, B))
        err = float((split_gemm(A, B) - torch.bmm(A.double(), B.double()).float()).abs().max())
        print(f'Co {Co:4d} Ci {Ci:4d} P {P:6d}: bmm {t_bmm:7.3f} ms ({fl / t_bmm / 1e9:6.1f} TF)  '
              f'split16 {t_split:7.3f} ms ({fl / t_split / 1e9:6.1f} TF)  max|err| {err:.2e}', flush=True)


if __name__ == '__main__':
    main()
