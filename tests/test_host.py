"""Host-side logic of the drop-in boundary (no GPU): configuration mirroring the reference's
globals, loud failure on CPU tensors (no silent CPU fallback), unsupported variants."""

import pytest
import torch

import nfi
from nfi import ops


def _field(dev='cpu'):
    return nfi.TriplaneField(planes=torch.zeros(1, 3, 32, 8, 8), palette=torch.zeros(1, 10, 3),
                             w1=torch.zeros(64, 32), b1=torch.zeros(64), w2=torch.zeros(11, 64),
                             b2=torch.zeros(11))


def test_configure_from_reference_globals():
    class A:
        fine_sampling = True
        use_sdf = True
        attention_values = 10
        use_viewdir = False
    cfg = nfi.configure(args=A(), dataset_config={'scene_range': 0.55, 'white_background': True})
    assert cfg.scene_range == 0.55 and cfg.white_background and cfg.fine_sampling
    nfi.configure(scene_range=1.4, white_background=False)


def test_cpu_tensors_fail_loudly():
    cam = torch.eye(4).unsqueeze(0)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        nfi.render(_field(), 8, 8, cam, torch.ones(1), None, None, None, 32)


def test_normals_need_sdf_field():
    nfi.configure(use_sdf=False)
    try:
        with pytest.raises(ValueError, match='SDF'):
            nfi.render(_field(), 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32,
                       compute_normals=True)
    finally:
        nfi.configure(use_sdf=True)


def test_field_heads_follow_the_field():
    """attention_values 0 / use_sdf False fields: normals need the SDF (generator.py:600-601),
    semantics the attention values (:670-671); the checks fire before any device work."""
    f = _field()
    f.use_sdf = False
    with pytest.raises(ValueError, match='SDF'):
        nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32, compute_normals=True)
    f = _field()
    f.attention_values, f.palette = 0, None
    with pytest.raises(ValueError, match='attention'):
        nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32, compute_semantics=True)
    with pytest.raises(RuntimeError, match='HIP devices only'):       # and the rest reaches the op
        nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)


def test_viewdir_config_must_match_the_field():
    """--use_viewdir without a mapper in the generator (or the reverse) is rejected up front (the
    reference would fail inside the sampler, generator.py:464-465, 661-663)."""
    nfi.configure(use_viewdir=True)
    try:
        with pytest.raises(ValueError, match='use_viewdir'):
            nfi.render(_field(), 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)
    finally:
        nfi.configure(use_viewdir=False)
    f = _field()
    f.viewdir_mapper = torch.nn.Identity()
    with pytest.raises(ValueError, match='use_viewdir'):
        nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)


def test_frozen_decoder_required():
    f = _field()
    f.w1.requires_grad_()
    with pytest.raises(NotImplementedError, match='frozen'):
        nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)


def test_trainable_viewdir_output_layer_refused():
    """The view-direction mapper's output layer is packed into the kernels' head: a trainable one
    would get no gradient, so render() refuses it (the trunk may still train)."""
    from nfi.viewdir import ViewDirectionMapper
    f = _field()
    f.viewdir_mapper = ViewDirectionMapper(10)
    f.viewdir_mapper.requires_grad_(False)
    f.viewdir_mapper.output.weight.requires_grad_()
    nfi.configure(use_viewdir=True)
    try:
        with pytest.raises(NotImplementedError, match='viewdir_mapper.output.weight'):
            nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)
        f.viewdir_mapper.output.weight.requires_grad_(False)
        with torch.no_grad(), pytest.raises(RuntimeError, match='HIP devices only'):
            f.viewdir_mapper.output.weight.requires_grad_()
            nfi.render(f, 8, 8, torch.eye(4)[None], torch.ones(1), None, None, None, 32)   # no_grad: allowed
    finally:
        nfi.configure(use_viewdir=False)


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py --gpus N without torchrun starts N rank processes itself, and refuses (before any
    GPU work) when fewer than N GPUs are visible: it never reports a smaller run under n_gpus N."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1'],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert 'needs 2 visible GPUs' in r.stderr
    assert r.stdout.strip() == ''


def test_planes_shape_checked():
    with pytest.raises(RuntimeError):
        ops.planes_texel_major(torch.zeros(1, 3, 32, 8, 8))


def test_dense_view_check():
    # planes_texel_major keeps a channels_last view only when it is dense (d planes are written
    # with the view's strides into zeros_like(view)); sliced buffers must take the copy path
    cl = torch.zeros(4, 96, 8, 8).to(memory_format=torch.channels_last)
    tm = cl.view(4, 3, 32, 8, 8).permute(0, 1, 3, 4, 2)
    assert ops._dense(tm)
    assert torch.zeros_like(tm).stride() == tm.stride()
    assert not ops._dense(cl[::2].view(2, 3, 32, 8, 8).permute(0, 1, 3, 4, 2))
    cl128 = torch.zeros(2, 128, 8, 8).to(memory_format=torch.channels_last)
    assert not ops._dense(cl128[:, :96].view(2, 3, 32, 8, 8).permute(0, 1, 3, 4, 2))


def test_stage_seams_refuse_cpu_tensors():
    """nfi.stages (the per-stage seams) run on HIP devices only, like render()."""
    from nfi import stages
    ro, rd = torch.zeros(4, 3), torch.ones(4, 3)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        stages.compute_near_far_planes(ro, rd, 1.4)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        stages.sample_pdf(torch.zeros(4, 9), torch.zeros(4, 8), 8)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        stages.render_volume_density(torch.zeros(4, 8), torch.zeros(4, 8, 3), ro, rd, torch.zeros(4, 8))
    with pytest.raises(RuntimeError, match='HIP devices only'):
        stages.make_sampler(_field())(torch.zeros(1, 5, 3))


def test_split_f16_products_carry_fp32_error():
    """The arithmetic of the split-f16 decoder (nfi_render.hip), emulated in numpy:
    operands scaled by a power of two (largest |v| in [2^14, 2^15)), split as hi = f16(v),
    lo = f16(v - hi); a contraction is lo.hi + hi.lo + hi.hi with exact products accumulated in
    fp32.  Its error against fp64, relative to sum |a b|, matches an fp32 dot product's at operand
    magnitudes 1e-5 .. 1e3 (the per-wave / per-matrix scaling keeps every value in fp16's normal
    range); without the scaling, small operands lose that accuracy."""
    import numpy as np

    def scale(a, axis=None):
        m = np.max(np.abs(a), axis=axis, keepdims=True)
        e = 15 - np.frexp(np.where(m > 0, m, 1.0))[1]
        return np.ldexp(np.float32(1), e).astype(np.float32)

    def split(a):
        h = a.astype(np.float16)
        return h, (a - h.astype(np.float32)).astype(np.float16)

    def split_mm(W, X, sw, sx):
        wh, wl = split(W * sw)
        xh, xl = split(X * sx)
        f = lambda p, q: p.astype(np.float32) @ q.astype(np.float32)   # f16 x f16 products: exact in fp32
        return (f(wl, xh) + f(wh, xl) + f(wh, xh)) / (sw * sx)

    rng = np.random.default_rng(0)
    W = (rng.standard_normal((64, 32)) / np.sqrt(32)).astype(np.float32)
    for mag in (1e-5, 1e-2, 1.0, 1e3):
        X = (rng.standard_normal((32, 512)) * mag).astype(np.float32)
        ref = W.astype(np.float64) @ X.astype(np.float64)
        den = np.abs(W).astype(np.float64) @ np.abs(X).astype(np.float64)
        e32 = np.max(np.abs((W @ X).astype(np.float64) - ref) / den)
        es = np.max(np.abs(split_mm(W, X, scale(W), scale(X, axis=0)) - ref) / den)
        assert es <= 4 * e32 + 1e-7, (mag, es, e32)
    # unscaled small operands fall into fp16 subnormals: far from fp32 accuracy
    X = (rng.standard_normal((32, 512)) * 1e-5).astype(np.float32)
    ref = W.astype(np.float64) @ X.astype(np.float64)
    den = np.abs(W).astype(np.float64) @ np.abs(X).astype(np.float64)
    assert np.max(np.abs(split_mm(W, X, np.float32(1), np.float32(1)) - ref) / den) > 1e-4


def test_split_gemm_host_rules():
    """Host rules around the split-f16 GEMM (nfi/conv.py): the K split covers the CUs about twice
    for few output tiles and never splits below 8 K-steps of 32; the fused Winograd kernel is kept
    for 64 -> 64 layers only while the split GEMM is on; a weight set carries its per-stream maxima
    buffers."""
    from nfi import conv
    assert conv.ksplit(600, 512) == 1 and conv.ksplit(512, 4608) == 1
    assert conv.ksplit(4, 4608) == 18 and conv.ksplit(32, 2304) == 9 and conv.ksplit(144, 512) == 2
    assert conv.ksplit(8, 256) == 1                        # K // 256: never below 8 K-steps of 32
    for tiles in (1, 7, 100, 511):
        for K in (256, 512, 1152, 4608):
            k = conv.ksplit(tiles, K)
            assert 1 <= k <= max(1, K // 256) and (k == 1 or tiles * k >= min(512, tiles * (K // 256)))
    ws = conv.WeightSet(torch.zeros(36, 64, 64), torch.zeros(1), None)
    old = conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO, conv.SPLIT16
    try:
        conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO, conv.SPLIT16 = True, 64, 64, True
        assert conv._fused_ok(ws, 64, 64) and not conv._fused_ok(ws, 64, 128) and not conv._fused_ok(ws, 128, 64)
        conv.SPLIT16 = False                               # hipBLASLt products: the round-3 rule (Ci only)
        assert conv._fused_ok(ws, 64, 128)
        assert not conv._fused_ok(conv.WeightSet(ws.U, None, None), 64, 64)   # no packed operands
    finally:
        conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO, conv.SPLIT16 = old
    assert ws.vmax == {}
