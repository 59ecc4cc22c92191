"""The deterministic backward (nfi_set_deterministic / nfi.ops.DETERMINISTIC /
torch.use_deterministic_algorithms): tile bins sorted by sample index, d planes summed from per-chunk
partial tile images in a fixed order instead of float atomics.  Two runs must agree bit for bit, the
results must pass the same parity bounds as the atomics form (tests/test_gpu_parity.py's check), and
the two forms must agree to fp32 summation-order rounding.  (The reference's grid_sample backward
itself accumulates with atomics: it has no deterministic form to compare against.)"""

import pytest
import torch

import bench
import nfi
from golden_io import load
from gpu_helpers import rel_l2, run_hip, run_oracle, run_oracle64
from nfi import _lib, ops
from test_gpu_parity import check

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


@pytest.fixture
def det_mode():
    prev = ops.DETERMINISTIC
    yield
    ops.DETERMINISTIC = prev
    _lib.load().nfi_set_deterministic(0)


@pytest.mark.parametrize('case', ['p3d', 'shapenet'])
def test_deterministic_golden_bitwise_and_parity(case, det_mode):
    d, meta = load(f'render_{case}')
    ops.DETERMINISTIC = True
    a = run_hip(d, meta, DEV)
    b = run_hip(d, meta, DEV)
    for key in a:
        assert torch.equal(a[key], b[key]), f'{key} differs between two deterministic runs'
    check(a, run_oracle(d, meta), run_oracle64(d, meta))
    ops.DETERMINISTIC = False
    c = run_hip(d, meta, DEV)
    assert rel_l2(a['d_planes'], c['d_planes']) < 1e-5


def _full_step(det, seed=0):
    cfg = list(bench.CONFIGS['p3d_fwdbwd'])
    cfg[3] = 2                                    # B = 2 images at the full 128^2, 64 + 64 samples
    cfg = tuple(cfg)
    nfi.configure(scene_range=cfg[0], white_background=cfg[1], fine_sampling=True)
    batch = bench.make_inputs(cfg, DEV, seed)
    ops.DETERMINISTIC = det
    torch.manual_seed(1234)                       # (the render's Philox seed is drawn from torch's generator)
    bench.run_step(nfi, batch, cfg, True)
    torch.cuda.synchronize()
    return batch['field'].planes.grad.clone(), batch['field'].palette.grad.clone()


def test_deterministic_full_size(det_mode):
    p1, q1 = _full_step(True)
    p2, q2 = _full_step(True)
    assert torch.equal(p1, p2) and torch.equal(q1, q2)
    p3, _ = _full_step(False)
    assert rel_l2(p1, p3) < 1e-5


def test_follows_torch_deterministic_algorithms(det_mode):
    """ops.DETERMINISTIC None: torch.use_deterministic_algorithms(True) selects the deterministic form
    (set in the thread that runs the backward: autograd's device thread)."""
    prev = torch.are_deterministic_algorithms_enabled()
    lib = _lib.load()
    before = lib.nfi_set_deterministic(-1)             # this (the caller's) thread's setting
    torch.use_deterministic_algorithms(True, warn_only=True)
    seen = []
    try:
        for _ in range(2):
            ops.DEBUG_BACKWARD = {}
            p, _ = _full_step(None)
            seen.append(ops.DEBUG_BACKWARD.get('deterministic'))
            if len(seen) == 1:
                p1 = p
            else:
                p2 = p
    finally:
        ops.DEBUG_BACKWARD = None
        torch.use_deterministic_algorithms(prev)
    # the mode was in effect on the thread that ran each backward (autograd's device thread), and the
    # caller's thread setting is untouched (nfi_set_deterministic is per host thread, include/nfi.h)
    assert seen == [1, 1], seen
    assert lib.nfi_set_deterministic(-1) == before
    assert torch.equal(p1, p2)
