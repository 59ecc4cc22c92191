"""The Winograd batched GEMMs (36 products [Co x Ci] x [Ci x P]) on hipBLASLt in the four operand
layouts (V as [36][Ci][P] or [36][P][Ci]; M as [36][Co][P] or [36][P][Co]) on the LPIPS-VGG and
synthesis shapes: which layout should the transforms produce?  Usage (GPU box):
python scripts/wino_gemm_layouts.py"""
import torch

SHAPES = [(128, 128, 16384), (256, 128, 4096), (256, 256, 4096), (512, 256, 1024), (512, 512, 1024),
          (512, 512, 256), (64, 128, 16384), (128, 64, 16384)]


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
    dev = torch.device('cuda:0')
    for co, ci, p in SHAPES:
        U = torch.randn(36, co, ci, device=dev)
        V = torch.randn(36, ci, p, device=dev)
        Vt = V.transpose(1, 2).contiguous()            # [36][P][Ci]
        Ut = U.transpose(1, 2).contiguous()            # [36][Ci][Co]
        gf = 2 * 36 * co * ci * p / 1e9
        res = {
            'M=UV (V ci-major)': timeit(lambda: torch.bmm(U, V)),
            'M=UV (V p-major)': timeit(lambda: torch.bmm(U, Vt.transpose(1, 2))),
            'Mt=VtUt (V p-major, M p-major)': timeit(lambda: torch.bmm(Vt, Ut)),
            'Mt=VtUt (V ci-major, M p-major)': timeit(lambda: torch.bmm(V.transpose(1, 2), Ut)),
        }
        print(f'Co={co:3d} Ci={ci:3d} P={p:5d}: ' + '  '.join(f'{k} {gf / v:5.0f} TF' for k, v in res.items()),
              flush=True)


if __name__ == '__main__':
    main()
