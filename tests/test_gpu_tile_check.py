"""The tile pass under its integrity-check build (nfi_render.hip NFI_TILE_CHECK).

`libnfi_hip_tilecheck.so` (built by __graft_entry__.build / `nfi/build.py --variant=tilecheck`) is the
product sources with -DNFI_TILE_CHECK=1: the tile pass checks every global index it derives from
loaded or shuffled data (rows, records, chunk / tile ranges), that every bin list is complete
(cursor == offsets + counts after the field backward's append), reads back each LDS stage it writes
(texels, gradient rows against gfeat, the wave-image dump), compares each scalar entry record with
the vector one, and sums d planes a second way (per-entry float atomics straight from the list and
gfeat) against the register-image sums; any violation fails the backward with NFI_ECHECK and the
first failure's code / chunk / tile / lane.  A child process loads it through NFI_LIBRARY and renders
the cases that exposed round 4's padded-layout failure (R = 64 planes, 16 x 16 rays, 64 + 64 samples,
both binning paths) and the full plane resolution, each against the fp64 oracle's bounds."""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'nerf-from-image_amd', 'nfi', 'libnfi_hip_tilecheck.so')

WORKER = r'''
import os, sys
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, 'tests'), root, os.path.join(root, 'nerf-from-image_amd')]
import torch
from nfi import _lib, ops
assert os.path.samefile(_lib.LIB_PATH, os.environ['NFI_LIBRARY'])
from gpu_helpers import rel_l2, run_hip, run_oracle, run_oracle64, synthetic_inputs
dev = torch.device('cuda:0')
cases = [dict(B=2, H=16, W=16, S=64, R=64, seed=40), dict(B=2, H=16, W=16, S=64, R=64, seed=21),
         dict(B=1, H=24, W=24, S=64, R=256, seed=5)]
for c in cases:
    inp, meta = synthetic_inputs(scene_range=1.4, **c)
    outs = []
    for fwd_counts in (True, False):
        ops.FORWARD_TILE_COUNTS = fwd_counts
        outs.append(run_hip(inp, meta, dev))          # raises NfiError on any violated check
    ops.FORWARD_TILE_COUNTS = True
    assert rel_l2(outs[0]['d_planes'], outs[1]['d_planes']) < 1e-5
    r32, r64 = run_oracle(inp, meta), run_oracle64(inp, meta)
    for key, floor in (('d_planes', 1e-3), ('d_palette', 1e-4), ('d_cam', 1e-4)):
        e_hip, e_ref = rel_l2(outs[0][key], r64[key]), rel_l2(r32[key], r64[key])
        assert e_hip <= max(floor, 4 * e_ref), (c, key, e_hip, e_ref)
    print('case ok', c, flush=True)
print('tile check ok', flush=True)
'''


def test_tile_pass_integrity_checks(tmp_path):
    assert os.path.exists(LIB), f'{LIB} missing: build it with python nerf-from-image_amd/nfi/build.py --variant=tilecheck'
    script = tmp_path / 'worker.py'
    script.write_text(WORKER)
    env = dict(os.environ, NFI_LIBRARY=LIB)
    p = subprocess.run([sys.executable, str(script), ROOT], env=env, timeout=240, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert 'tile check ok' in p.stdout
