"""Split-f16 GEMM (nfi_gemm_split16) vs torch.bmm (hipBLASLt fp32) on the Winograd products of the
inversion step (36 batched [Co x Ci] x [Ci x P]): ms and TFLOP/s (fp32-equivalent, 2 M N K per
product) per shape, the GEMM launch alone (A split and B's maximum computed beforehand, as the
Winograd path does: weights split once, the maximum left by the input transform); both kernels of
the entry (default: the general one; NFI_GEMM_KERNEL=2: the wide-load one).  Then the up-sampling
convolutions' shared-A GEMMs (W9 x per image, W9^T dP; conv.split_matmul_shared incl. the maximum
pass and the K split) against torch.matmul.  GPU box: python scripts/gemm_bench.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd')]
import torch  # noqa: E402

from nfi import _lib, conv  # noqa: E402

DEV = torch.device('cuda:0')
# (Co, Ci, P): LPIPS VGG16 trunk at 128^2 over 4 images x 16 copies (P = 64 (H/4)^2), producer 3x3
# layers at B = 4 (P = 4 (H/4)^2)
SHAPES = [(128, 128, 16384), (256, 128, 4096), (256, 256, 4096), (512, 256, 1024), (512, 512, 1024),
          (512, 512, 256), (256, 256, 16384), (128, 128, 65536), (512, 512, 4096), (96, 96, 4100)]


# tile:xcd:prefetch variants of the general kernel (NFI_GEMM_TILE, NFI_GEMM_XCD, NFI_GEMM_PF)
VARIANTS = [v.split(':') for v in os.environ.get('GEMM_VARIANTS', '22:0:1 22:1:1 22:0:2 22:1:2').split()]


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


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
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    for Co, Ci, P in SHAPES:
        A = torch.randn((36, Co, Ci), device=DEV)
        B = torch.randn((36, Ci, P), device=DEV)
        hi = torch.empty(A.shape, device=DEV, dtype=torch.int16)
        lo = torch.empty(A.shape, device=DEV, dtype=torch.int16)
        inv = torch.empty((36,), device=DEV)
        slots = torch.empty((int(lib.nfi_split16_slot_words()),), device=DEV, dtype=torch.int32)   # per-image maxima + counter
        t_pack = timeit(lambda: _lib.check(lib.nfi_split16_pack(_p(A), 36, Co * Ci, _p(hi), _p(lo), _p(inv), st), 'pack'))
        _lib.check(lib.nfi_absmax_slots(_p(B), 1, B.numel(), _p(slots), st), 'absmax')
        C = torch.empty((36, Co, P), device=DEV)
        gemm = lambda: _lib.check(lib.nfi_gemm_split16(_p(hi), _p(lo), _p(inv), _p(B), _p(slots), _p(C), 36, Co, P, Ci, P, st),
                                  'gemm')
        fl = 2 * 36 * Co * Ci * P
        ref = torch.bmm(A.double(), B.double()).float()
        t_bmm = timeit(lambda: torch.bmm(A, B))
        res = []
        for tile, xcd, pf in VARIANTS:
            os.environ['NFI_GEMM_TILE'] = tile
            os.environ['NFI_GEMM_XCD'] = xcd
            os.environ['NFI_GEMM_PF'] = pf
            C.zero_()
            t = timeit(gemm)
            err = float((C - ref).abs().max())
            res.append(f't{tile}x{xcd}p{pf} {t:6.3f} ms ({fl / t / 1e9:5.1f} TF{", err %.0e" % err if err > 2e-4 else ""})')
        for k in ('NFI_GEMM_TILE', 'NFI_GEMM_XCD', 'NFI_GEMM_PF'):
            os.environ.pop(k)
        mb = 36 * (Ci + Co) * P * 4 / 1e6
        print(f'Co {Co:4d} Ci {Ci:4d} P {P:6d} ({mb:5.0f} MB): bmm {t_bmm:7.3f} ms ({fl / t_bmm / 1e9:6.1f} TF)  '
              + '  '.join(res) + f'  pack {t_pack:.3f} ms', flush=True)

    # up-sampling layers of the 256^2 producer at B = 4: (M, N, K) forward W9 x and backward W9^T dP
    for M, N, K in [(4608, 16, 512), (4608, 64, 512), (4608, 256, 512), (4608, 1024, 512), (2304, 4096, 512),
                    (1152, 16384, 256), (512, 16, 4608), (512, 64, 4608), (512, 256, 4608), (512, 1024, 4608),
                    (512, 4096, 2304), (256, 16384, 1152)]:
        A = torch.randn((M, K), device=DEV) / K ** 0.5
        X = torch.randn((4, K, N), device=DEV)
        As = conv.split_matrix(A)
        t_mm = timeit(lambda: torch.matmul(A, X))
        t_sp = timeit(lambda: conv.split_matmul_shared(As, X))
        err = float((conv.split_matmul_shared(As, X) - torch.matmul(A.double(), X.double())).abs().max())
        ks = conv.ksplit(4 * -(-M // 128) * -(-N // 128), K)
        fl = 2 * 4 * M * N * K
        print(f'shared M {M:5d} N {N:6d} K {K:5d}: matmul {t_mm:7.3f} ms ({fl / t_mm / 1e9:6.1f} TF)  split {t_sp:7.3f} ms '
              f'({fl / t_sp / 1e9:6.1f} TF, ksplit {ks}, err {err:.1e})', flush=True)


if __name__ == '__main__':
    main()
