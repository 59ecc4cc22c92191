"""Property tier: hypothesis draws render configurations — batch, non-square image
sizes, samples per ray, plane resolution, scene range, orthographic / perspective cameras, white
background, deterministic / randomized sampling, fine sampling on / off, seeds — and every draw
must (a) match the oracle under the parity bar of tests/test_gpu_parity.py and (b) keep the
compositing invariants: 0 <= mask <= 1 (sum of weights of a transmittance product), rgb within
the palette's range (+ the white background), depth within [0, far], merged sample depths
ascending and inside [near, far], finite gradients."""

import pytest
import torch
from hypothesis import HealthCheck, given, settings, strategies as st

from gpu_helpers import run_hip, run_oracle, run_oracle64, synthetic_inputs
from test_gpu_parity import check

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


@st.composite
def configs(draw):
    return dict(B=draw(st.integers(1, 2)), H=draw(st.integers(3, 10)), W=draw(st.integers(3, 10)),
                S=draw(st.sampled_from([4, 7, 16, 33, 64, 65])), R=draw(st.sampled_from([8, 16, 33])),
                scene_range=draw(st.sampled_from([0.55, 1.4, 2.0])), ortho=draw(st.booleans()),
                white_bg=draw(st.booleans()), randomize=draw(st.booleans()), fine=draw(st.booleans()),
                seed=draw(st.integers(0, 10_000)))


@settings(max_examples=60, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=configs())
def test_random_configurations_match_oracle_and_invariants(cfg):
    fine = cfg.pop('fine')
    inp, meta = synthetic_inputs(**cfg)
    meta['fine'] = int(fine)
    dbg = {}
    hip = run_hip(inp, meta, DEV, debug=dbg)
    check(hip, run_oracle(inp, meta), run_oracle64(inp, meta))
    eps = 1e-5
    mask, rgb, depth = hip['mask'], hip['rgb'], hip['depth']
    assert float(mask.min()) >= -eps and float(mask.max()) <= 1 + eps
    lo, hi = -1.002 - eps, 1.002 + eps + (1.0 if cfg['white_bg'] else 0.0)   # palette range
    assert float(rgb.min()) >= lo and float(rgb.max()) <= hi
    near, far = dbg['near'].reshape(-1, 1).cpu(), dbg['far'].reshape(-1, 1).cpu()
    assert bool((near <= far).all())
    assert float(depth.min()) >= -eps and bool((depth.reshape(-1, 1) <= far + 1e-4).all())
    t = dbg['t_sorted'].cpu()
    assert bool((t[:, 1:] >= t[:, :-1]).all())
    span = far - near
    assert bool((t >= near - 1e-5 * span).all()) and bool((t <= far + 1e-5 * span).all())
    for k in ('d_planes', 'd_palette', 'd_cam', 'd_focal'):
        if k in hip:
            assert bool(torch.isfinite(hip[k]).all()), k
