"""The forward's tap gather alone (scripts/ubench/gather_probe.hip: the product's gather_features
over the forward's own merged sample depths, at the forward's occupancy, nothing else in the
kernel) against the full forward launch, on bench.py's p3d_fwdbwd inputs (B=8, 128², 64+64).
Gives the measured floor the tap stream sets for render_fwd.
Usage (GPU box, after building the probe library, see the .hip header): python scripts/gather_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import ops  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    cfg = bench.CONFIGS['p3d_fwdbwd']
    sr, wbg, flipped, B, H, S, pose, bwd = cfg
    nfi.configure(scene_range=sr, white_background=wbg, fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 1)
    f = batch['field']
    dbg = {}
    with torch.no_grad():
        nfi.render(f, H, H, batch['cam'], batch['focal'], None, None, None, S, randomize=True, debug=dbg)
    torch.cuda.synchronize()
    args = dbg['args']
    tensors = dbg['args_tensors']   # (the tensors args points at stay referenced while it is used)
    N = 2 * S
    n = B * H * H
    out = torch.empty((n * N,), device=dev)
    lib = ctypes.CDLL(os.environ.get('NFI_PROBE_LIB') or os.path.join(ROOT, 'scripts', 'ubench', 'libgather_probe.so'))
    lib.nfi_gather_probe.restype = ctypes.c_int32
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def probe():
        assert lib.nfi_gather_probe(ctypes.byref(args), ctypes.c_void_p(out.data_ptr()), stream) == 0

    def render():
        with torch.no_grad():
            nfi.render(f, H, H, batch['cam'], batch['focal'], None, None, None, S, randomize=True)

    res = {}
    for name, fn in (('gather_only', probe), ('forward_no_grad', render)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / reps, 4)
    samples = n * N
    res['samples'] = samples
    res['tap_bytes'] = samples * 1536
    res['gather_only_tap_TBps'] = round(samples * 1536 / (res['gather_only'] * 1e-3) / 1e12, 2)
    res['checksum_finite'] = bool(torch.isfinite(out).all())
    del tensors
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
