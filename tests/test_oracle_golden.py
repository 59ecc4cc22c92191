"""Pin the CPU oracle (oracle/render_oracle.py) to the reference's golden vectors.

The fixtures were produced by the reference's own code (tests/golden/gen_golden.py); the
oracle restates that code op for op, so forward outputs and gradients must agree to fp32
rounding of identical op graphs (in practice bit-exact).
"""

import pytest
import torch

from golden_io import EXTRAS_CASES, RENDER_CASES, VARIANT_CASES, VIEWDIR_CASES, ZBUFFER_CASES, field_from, load
from oracle import render_oracle as orc


def _run_oracle(d, meta):
    field = field_from(d, meta)
    field.planes = field.planes.clone().requires_grad_()
    if field.palette is not None:
        field.palette = field.palette.clone().requires_grad_()
    ncg = bool(meta['force_no_cam_grad'])
    cam = d['cam'].clone().requires_grad_(not ncg)
    focal = d.get('focal')
    if focal is not None:
        focal = focal.clone().requires_grad_(not ncg)
    rgb, depth, mask = orc.render(field, meta['H'], meta['W'], cam, focal, d.get('center'),
                                  d.get('bbox'), meta['S'], randomize=bool(meta['randomize']),
                                  white_background=bool(meta['white_bg']),
                                  force_no_cam_grad=ncg, u_coarse=d['u_coarse'],
                                  u_fine=d['u_fine'], zbuffer=bool(meta.get('zbuffer', 0)))
    loss = (rgb * d['g_rgb']).sum() + (mask * d['g_mask']).sum()
    loss.backward()
    return rgb, depth, mask, field, cam, focal


@pytest.mark.parametrize('case', RENDER_CASES + VARIANT_CASES + VIEWDIR_CASES + ZBUFFER_CASES)
def test_oracle_render_matches_reference(case):
    d, meta = load(f'render_{case}')
    rgb, depth, mask, field, cam, focal = _run_oracle(d, meta)
    tol = dict(rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rgb.detach(), d['rgb'], **tol)
    torch.testing.assert_close(depth.detach(), d['depth'], **tol)
    torch.testing.assert_close(mask.detach(), d['mask'], **tol)
    torch.testing.assert_close(field.planes.grad, d['d_planes'], **tol)
    if 'd_palette' in d:
        torch.testing.assert_close(field.palette.grad, d['d_palette'], **tol)
    if 'd_cam' in d:
        torch.testing.assert_close(cam.grad, d['d_cam'], rtol=1e-5, atol=1e-5)
    if 'd_focal' in d:
        torch.testing.assert_close(focal.grad, d['d_focal'], rtol=1e-5, atol=1e-5)


def test_oracle_near_far_matches_reference():
    d, _ = load('stages')
    near, far = orc.compute_near_far_planes(d['nf_ro'], d['nf_rd'], 1.4)
    assert torch.equal(near, d['nf_near'])
    assert torch.equal(far, d['nf_far'])


def test_oracle_sample_pdf_matches_reference():
    d, _ = load('stages')
    S = d['pdf_bins'].shape[-1] + 1
    det = orc.sample_pdf(d['pdf_bins'], d['pdf_w'], S, deterministic=True)
    rnd = orc.sample_pdf(d['pdf_bins'], d['pdf_w'], S, deterministic=False, u=d['pdf_u'])
    assert torch.equal(det, d['pdf_det'])
    assert torch.equal(rnd, d['pdf_rnd'])


@pytest.mark.parametrize('case', EXTRAS_CASES)
def test_oracle_eval_outputs_match_reference(case):
    """compute_normals / compute_semantics / compute_coords (run.py:227-257, 293-335)."""
    d, meta = load(f'render_{case}')
    field = field_from(d, meta)
    rgb, depth, mask, nmap, smap = orc.render(
        field, meta['H'], meta['W'], d['cam'], d['focal'], None, None, meta['S'], randomize=True,
        white_background=bool(meta['white_bg']), force_no_cam_grad=True, u_coarse=d['u_coarse'],
        u_fine=d['u_fine'], compute_normals=bool(meta['compute_normals']),
        compute_semantics=bool(meta['compute_semantics']), compute_coords=bool(meta['compute_coords']))
    tol = dict(rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rgb.detach(), d['rgb'], **tol)
    torch.testing.assert_close(depth.detach(), d['depth'], **tol)
    torch.testing.assert_close(mask.detach(), d['mask'], **tol)
    if 'normals' in d:
        torch.testing.assert_close(nmap.detach(), d['normals'], **tol)
    else:
        assert nmap is None
    if 'semantics' in d:
        torch.testing.assert_close(smap.detach(), d['semantics'], **tol)
    else:
        assert smap is None


def test_oracle_seams():
    """The oracle's restatements of the nerf_utils seams (cumprod_exclusive, get_ray_bundle,
    compute_query_points_from_rays, render_volume_density_weights_only) against the reference's
    own outputs and input gradients (tests/golden/seams.npz, fp32): the same op graphs, so equal
    to fp32 rounding (in practice bit for bit)."""
    d, _ = load('seams')

    def close(a, b, tol=1e-6):
        torch.testing.assert_close(a.detach(), b, rtol=tol, atol=tol)

    x = d['cp_x'].clone().requires_grad_()
    out = orc.cumprod_exclusive(x)
    (out * d['cp_g']).sum().backward()
    close(out, d['cp_out32'])
    close(x.grad, d['cp_dx32'], 1e-5)
    for tag in ('p', 'pcb', 'ob'):
        cam = d[f'rb{tag}_cam'].clone().requires_grad_()
        focal = d[f'rb{tag}_focal'].clone().requires_grad_() if f'rb{tag}_focal' in d else None
        ro, rd = orc.get_ray_bundle(6, 8, focal, cam, d.get(f'rb{tag}_bbox'), d.get(f'rb{tag}_center'))
        assert torch.equal(ro.detach(), d[f'rb{tag}_ro32']) and torch.equal(rd.detach(), d[f'rb{tag}_rd32'])
        ((ro * d[f'rb{tag}_gro']).sum() + (rd * d[f'rb{tag}_grd']).sum()).backward()
        close(cam.grad, d[f'rb{tag}_dcam32'], 1e-5)
        if focal is not None:
            close(focal.grad, d[f'rb{tag}_dfocal32'], 1e-5)
    for tag in ('d', 'r'):
        ro, rd = d['qp_ro'].clone().requires_grad_(), d['qp_rd'].clone().requires_grad_()
        S = d[f'qp{tag}_u'].shape[-1]
        pts, depth = orc.compute_query_points_from_rays(ro, rd, d['qp_near'], d['qp_far'], S, randomize=tag == 'r',
                                                        u=d[f'qp{tag}_u'])
        assert torch.equal(depth, d[f'qp{tag}_depth32']) and torch.equal(pts.detach(), d[f'qp{tag}_pts32'])
        (pts * d['qp_g']).sum().backward()
        close(ro.grad, d[f'qp{tag}_dro32'], 1e-5)
        close(rd.grad, d[f'qp{tag}_drd32'], 1e-5)
    sig, rdw, t = (d[k].clone().requires_grad_() for k in ('vw_sigma', 'vw_rd', 'vw_t'))
    w = orc.render_volume_density_weights_only(sig, torch.zeros_like(rdw), rdw, t)
    close(w, d['vw_w32'])
    (w * d['vw_g']).sum().backward()
    close(sig.grad, d['vw_dsigma32'], 1e-5)
    close(rdw.grad, d['vw_drd32'], 1e-5)
    close(t.grad, d['vw_dt32'], 1e-5)
