"""The TORCH_LIBRARY(nfi, ...) operators (csrc/nfi_torch.cpp, nfi/libnfi_torch.so): the C-ABI's
entry points as dispatcher ops, for callers that cannot go through ctypes — TorchScript (the
reference's nerf_utils functions are @torch.jit.script) and the C++ frontend.  Same kernels, same
arguments as nfi.ops / nfi.stages; load() fails loudly when the library is missing.

  torch.ops.nfi.rays(cam, focal, center, bbox, H, W, scene_range) -> (ro, rd, near, far)
  torch.ops.nfi.pack_decoder(w1, b1, w2, b2, attention_values=-1) -> dec
  torch.ops.nfi.volume_render(planes_tm, palette, ro, rd, near, far, dec, samples, fine,
                              white_background, randomize, scene_range, inv_alpha, beta, heads,
                              seed, u_coarse=None, u_fine=None) -> (rgb, depth, mask)
  torch.ops.nfi.volume_render_fwd / volume_render_bwd      the two halves (CUDA + Meta kernels)
  torch.ops.nfi.sample_pdf / compute_near_far_planes / cumprod_exclusive /
  render_volume_density_weights_only                        the nerf_utils seams
"""

from __future__ import annotations

import os

import torch

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
LIBRARY = os.path.join(HERE, 'libnfi_torch.so')
OPS = ('rays', 'pack_decoder', 'volume_render', 'volume_render_fwd', 'volume_render_bwd', 'sample_pdf',
       'compute_near_far_planes', 'cumprod_exclusive', 'render_volume_density_weights_only',
       'render_fwd', 'render_bwd', 'composite_fwd', 'composite_bwd', 'triplane_mlp_fwd', 'triplane_mlp_bwd')
_loaded = False


def load() -> None:
    """Register the operators (idempotent).  Raises NfiError when the library is missing."""
    global _loaded
    if _loaded:
        return
    if not os.path.exists(LIBRARY):
        raise _lib.NfiError(f'nfi: {LIBRARY} is missing: build it with python nerf-from-image_amd/nfi/build.py')
    _lib.load()                       # the C-ABI library it links (and the ABI check)
    torch.ops.load_library(LIBRARY)
    _loaded = True


def render_script_source() -> str:
    """A TorchScript-able render (run.py:193-348 without the producer): rays + fused volume render,
    for tests and callers that script their step.  render_rays draws its randomness from the Philox
    seed; render_rays_u takes the reference's draws (u_coarse / u_fine, or deterministic mode)."""
    return '''
def render_rays(planes_tm: torch.Tensor, palette: Optional[torch.Tensor], dec: torch.Tensor,
                cam: torch.Tensor, focal: Optional[torch.Tensor], H: int, W: int, S: int,
                scene_range: float, inv_alpha: float, beta: float, seed: int, white_background: bool):
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, H, W, scene_range)
    return torch.ops.nfi.volume_render(planes_tm, palette, ro, rd, near, far, dec, S, True,
                                       white_background, True, scene_range, inv_alpha, beta, 0, seed)


def render_rays_u(planes_tm: torch.Tensor, palette: Optional[torch.Tensor], dec: torch.Tensor,
                  cam: torch.Tensor, focal: Optional[torch.Tensor], H: int, W: int, S: int,
                  scene_range: float, inv_alpha: float, beta: float, white_background: bool,
                  randomize: bool, u_coarse: Optional[torch.Tensor], u_fine: Optional[torch.Tensor]):
    ro, rd, near, far = torch.ops.nfi.rays(cam, focal, None, None, H, W, scene_range)
    return torch.ops.nfi.volume_render(planes_tm, palette, ro, rd, near, far, dec, S, True,
                                       white_background, randomize, scene_range, inv_alpha, beta, 0, 0,
                                       u_coarse, u_fine)
'''
