"""Drop-in `render()` for run.py:176-350 on MI355X.

`render(target_model, height, width, tform_cam2world, focal_length, center, bbox, model_input,
depth_samples_per_ray, randomize=True, compute_normals=False, compute_semantics=False,
compute_coords=False, extra_model_outputs=[], extra_model_inputs={}, force_no_cam_grad=False)`
keeps the reference's signature, argument meaning and 6-tuple return
`(rgb, depth, mask, normals, semantics, model_outputs)`.  The reference reads the globals
`args` (use_viewdir, fine_sampling, use_sdf, attention_values) and `dataset_config`
(scene_range, white_background); here they come from `configure(args=..., dataset_config=...)`.

Everything from the camera to the composited pixel runs in the HIP kernels of
`nerf-from-image_amd/csrc` (see ops.py); the tri-plane producer (synthesis network) and
the palette producer (AttentionMapper) stay the caller's PyTorch modules.
"""

from __future__ import annotations

import types
from dataclasses import dataclass, field as dc_field
from typing import Any, Optional, Sequence

import torch

from . import ops
from .viewdir import viewdir_trunk


@dataclass
class RenderConfig:
    scene_range: float = 1.4
    white_background: bool = False
    fine_sampling: bool = True
    use_sdf: bool = True
    attention_values: int = 10
    use_viewdir: bool = False


_CONFIG = RenderConfig()


def configure(args: Any = None, dataset_config: Optional[dict] = None, **overrides) -> RenderConfig:
    """Set the reference's globals: `args` (arguments.py namespace) and `dataset_config`
    (loaders.get_dataset_config dict), or individual fields as keywords."""
    if args is not None:
        for k in ('fine_sampling', 'use_sdf', 'attention_values', 'use_viewdir'):
            if hasattr(args, k):
                setattr(_CONFIG, k, getattr(args, k))
    if dataset_config is not None:
        _CONFIG.scene_range = float(dataset_config['scene_range'])
        _CONFIG.white_background = bool(dataset_config['white_background'])
    for k, v in overrides.items():
        if not hasattr(_CONFIG, k):
            raise KeyError(k)
        setattr(_CONFIG, k, v)
    return _CONFIG


def get_config() -> RenderConfig:
    return _CONFIG


@dataclass
class TriplaneField:
    """The inputs the renderer reads from a Generator (generator.py:392-503)."""
    planes: torch.Tensor                 # [B,3,32,R,R] (contiguous or channels_last producer output)
    palette: Optional[torch.Tensor]      # [B,10,3] attention values (None: attention_values 0)
    w1: torch.Tensor                     # decoder.net[0].weight [64,32]
    b1: torch.Tensor                     # decoder.net[0].bias   [64]
    w2: torch.Tensor                     # decoder.net[2].weight [11,64] ([4,64] without attention)
    b2: torch.Tensor                     # decoder.net[2].bias   [11]
    alpha: float = 1.0                   # Generator.alpha (sigma = laplace_cdf / alpha)
    beta: float = 0.1                    # Generator.beta
    model_outputs: dict = dc_field(default_factory=dict)
    attention_values: int = 10           # Generator.attention_values (0: wide-sigmoid colour head)
    use_sdf: bool = True                 # Generator.use_sdf (False: softplus(d - 1) density)
    viewdir_mapper: Any = None           # Generator.viewdir_mapper (--use_viewdir; w2 is then [33,64])


def _as_float(x) -> float:
    return float(x.detach().reshape(-1)[0].item()) if torch.is_tensor(x) else float(x)


def _sdf_params(gen):
    """(alpha, beta) of a generator as floats, read from the device once per value: a cache keyed
    on the parameters' storage and in-place version counters, so the inversion loop does not
    synchronise the host on every render (the generator is frozen there)."""
    a, b = gen.alpha, gen.beta
    if not (torch.is_tensor(a) and torch.is_tensor(b)):
        return _as_float(a), _as_float(b)
    key = (a.data_ptr(), a._version, b.data_ptr(), b._version)
    cached = getattr(gen, '_nfi_sdf_params', None)
    if cached is None or cached[0] != key:
        cached = (key, (_as_float(a), _as_float(b)))
        try:
            object.__setattr__(gen, '_nfi_sdf_params', cached)
        except AttributeError:
            pass
    return cached[1]


def field_from_generator(gen, c, extra_model_outputs: Sequence[str] = (),
                         extra_model_inputs: Optional[dict] = None) -> TriplaneField:
    """Runs the parts of Generator.forward (generator.py:423-503) that produce the path's
    inputs — ws, AttentionMapper palette, synthesis tri-planes — on the reference's own
    modules: unconditional, no encoder, no viewdir; attention_values 10 (the inversion
    configuration) or 0, use_sdf or not, with or without the view-direction mapper (whose
    per-ray trunk render() runs on the rays, run.py:216-219)."""
    extra_model_inputs = extra_model_inputs or {}
    for k in extra_model_inputs:
        if k not in ('freeze_noise', 'attention_values', 'attention_values_bias'):
            raise AssertionError(k)
    if getattr(gen, 'use_encoder', False) or getattr(gen, 'num_classes', None):
        raise NotImplementedError('encoder-/class-conditioned generators are outside the inversion path')
    nattn = int(getattr(gen, 'attention_values', 0))
    use_sdf = bool(getattr(gen, 'use_sdf', False))
    if not 0 <= nattn <= MAX_ATTENTION:
        raise NotImplementedError(f'nfi renders fields with 0..{MAX_ATTENTION} attention values (got {nattn})')
    if c.dim() == 3:
        ws = c.expand(-1, gen.mapping_network.backbone.num_ws, -1).contiguous() if c.shape[1] == 1 else c
    else:
        ws = gen.mapping_network(c, None)
    if nattn:                           # generator.py:451-462
        assert ws.shape[1] == 15
        w_syn, w_tex = ws.split([14, 1], dim=1)     # one split (its backward is one cat)
        w_tex = w_tex[:, 0]
        if 'attention_values' in extra_model_inputs:
            palette = extra_model_inputs['attention_values']
        else:
            palette = gen.texture_mapper(w_tex)
            if 'attention_values_bias' in extra_model_inputs:
                palette = palette + extra_model_inputs['attention_values_bias']
    else:
        w_syn, palette = ws, None
    kw = {'noise_mode': 'const'} if extra_model_inputs.get('freeze_noise') else {}
    planes = gen.synthesis_network(w_syn, **kw)
    planes = planes.view(c.shape[0], 3, 32, planes.shape[-2], planes.shape[-1])
    outs = {}
    if 'attention_values' in extra_model_outputs and palette is not None:
        outs['attention_values'] = palette
    for k in extra_model_outputs:
        if k not in ('attention_values',):
            raise NotImplementedError(f'model output {k!r} (training regulariser) is outside the path')
    dec = gen.decoder.net
    alpha, beta = _sdf_params(gen) if use_sdf else (1.0, 0.1)
    return TriplaneField(planes=planes, palette=palette, w1=dec[0].weight, b1=dec[0].bias,
                         w2=dec[2].weight, b2=dec[2].bias, alpha=alpha, beta=beta,
                         model_outputs=outs, attention_values=nattn, use_sdf=use_sdf,
                         viewdir_mapper=gen.viewdir_mapper if getattr(gen, 'use_viewdir', False) else None)


def _resolve_field(target_model, model_input, extra_model_outputs, extra_model_inputs) -> TriplaneField:
    if isinstance(target_model, TriplaneField):
        return target_model
    if hasattr(target_model, 'nfi_field'):
        return target_model.nfi_field(model_input, extra_model_outputs, extra_model_inputs)
    if hasattr(target_model, 'synthesis_network') and hasattr(target_model, 'decoder'):
        return field_from_generator(target_model, model_input, extra_model_outputs, extra_model_inputs)
    raise TypeError('target_model must be a TriplaneField, provide nfi_field(), or be a '
                    'reference-style Generator (synthesis_network + decoder)')


MAX_ATTENTION = 10   # the kernels' attention head: 10 logits (nfi_common.h NA); fewer are padded


def attention_padded(f: TriplaneField):
    """(w2, b2, palette) of a field with N = 1..9 attention values (generator.py:363-402, 665-679 allow
    any N) padded to the kernels' 10: zero decoder rows and palette rows, and a bias of -1e30 on the
    padded logits, whose softmax terms exp(-1e30 - max) are then exactly 0 — the softmax over the N
    real logits, the colour, and every gradient (0 to the padded rows; the palette's own rows through
    the concatenation) are those of the N-value head.  N = 0 or 10: the field's own tensors."""
    n = int(f.attention_values)
    if n in (0, MAX_ATTENTION):
        return f.w2, f.b2, f.palette
    if not 0 < n < MAX_ATTENTION:
        raise NotImplementedError(f'nfi renders fields with 0..{MAX_ATTENTION} attention values (got {n})')
    pad = MAX_ATTENTION - n
    w2 = torch.cat([f.w2.detach(), f.w2.new_zeros((pad, f.w2.shape[1]))]) if f.viewdir_mapper is None else f.w2
    b2 = torch.cat([f.b2.detach(), f.b2.new_full((pad,), -1e30)]) if f.viewdir_mapper is None else f.b2
    pal = torch.cat([f.palette, f.palette.new_zeros((f.palette.shape[0], pad, 3))], dim=1)
    return w2, b2, pal


def _check_frozen(f: TriplaneField):
    if torch.is_grad_enabled():
        for name in ('w1', 'b1', 'w2', 'b2'):
            if getattr(f, name).requires_grad:
                raise NotImplementedError(
                    f'decoder parameter {name} requires grad: nfi differentiates the inversion '
                    f'path, where the generator is frozen (run.py:630-632); call requires_grad_(False)')
        # the view-direction mapper's output layer is packed into the kernels' head (its trunk
        # stays an autograd module): a trainable output layer would silently get no gradient
        vm = f.viewdir_mapper
        if vm is not None:
            for name in ('weight', 'bias'):
                p = getattr(getattr(vm, 'output', None), name, None)
                if p is not None and p.requires_grad:
                    raise NotImplementedError(
                        f'viewdir_mapper.output.{name} requires grad: the kernels take the mapper\'s '
                        f'output layer as a frozen head (its trunk may train); call '
                        f'viewdir_mapper.output.requires_grad_(False)')


def render(target_model, height, width, tform_cam2world, focal_length, center, bbox, model_input,
           depth_samples_per_ray, randomize=True, compute_normals=False, compute_semantics=False,
           compute_coords=False, extra_model_outputs=[], extra_model_inputs={},
           force_no_cam_grad=False, *, u_coarse=None, u_fine=None, seed=None, debug=None,
           depth_mode: str = 'ray'):
    """run.py:176-350.  Extra keyword-only arguments (not in the reference) inject the random
    draws for parity testing (`u_coarse` [B,H,W,S], `u_fine` [B*H*W,S]) or fix the Philox
    seed; `debug` (a dict) receives intermediate depths.  depth_mode 'zbuffer' returns the
    camera-space z depth of the perspective eval scripts' render copies instead of the ray
    distance (eval_nusc_persp.py:221-228; see render_zbuffer)."""
    if depth_mode not in ('ray', 'zbuffer'):
        raise ValueError("depth_mode must be 'ray' or 'zbuffer'")
    cfg = _CONFIG
    if compute_normals and not cfg.use_sdf:
        raise ValueError('compute_normals needs an SDF field (run.py:229)')
    if compute_semantics and cfg.attention_values <= 0:
        raise ValueError('compute_semantics needs attention values (run.py:232)')
    # run.py:334-335: the coords map takes the semantic map's place
    extras = (1 if compute_normals else 0) | (4 if compute_coords else (2 if compute_semantics else 0))
    f = _resolve_field(target_model, model_input, extra_model_outputs, extra_model_inputs)
    _check_frozen(f)
    if bool(cfg.use_viewdir) != (f.viewdir_mapper is not None):
        raise ValueError('args.use_viewdir and the generator\'s view-direction mapper disagree '
                         '(the reference requires both or neither, generator.py:464-465, 661-663)')
    if compute_normals and not f.use_sdf:
        raise ValueError('compute_normals needs an SDF field (generator.py:600-601)')
    if compute_semantics and not f.attention_values:
        raise ValueError('compute_semantics needs attention values (generator.py:670-671)')
    heads = ((ops.HEAD_RGB_SIGMOID if f.attention_values == 0 else 0)
             | (0 if f.use_sdf else ops.HEAD_NERF_DENSITY)
             | (ops.HEAD_VIEWDIR if f.viewdir_mapper is not None else 0))
    ro, rd, near, far = ops.rays(tform_cam2world, focal_length, center, bbox, height, width,
                                 cfg.scene_range)
    if debug is not None:
        debug.update(ro=ro.detach(), rd=rd.detach(), near=near, far=far)
    if force_no_cam_grad:
        # run.py:211-214 detaches query points and directions (the reference's fine points keep a
        # gradient path to ray origins; its callers of this mode run under no_grad)
        ro, rd = ro.detach(), rd.detach()
    xray = vhead = None
    if f.viewdir_mapper is not None:
        # run.py:216-219: viewdirs = the (unit, possibly detached) ray directions; the mapper's
        # per-ray trunk (generator.py:223-238) here, its per-sample closure in the kernels
        xray = viewdir_trunk(f.viewdir_mapper, rd.unsqueeze(-2)).squeeze(-2)
        vw, vb = f.viewdir_mapper.output.weight, f.viewdir_mapper.output.bias
        if 0 < f.attention_values < MAX_ATTENTION:
            # the mapper's output layer gives the N logits here: padded like the decoder rows below
            pad = MAX_ATTENTION - int(f.attention_values)
            vw = torch.cat([vw.detach(), vw.new_zeros((pad, vw.shape[1]))])
            vb = torch.cat([vb.detach(), vb.new_full((pad,), -1e30)])
        vhead = ops.pack_viewdir_head(vw, vb)
    planes_tm = ops.planes_texel_major(f.planes)
    w2, b2, palette = attention_padded(f)
    dec = ops.pack_decoder(f.w1, f.b1, w2, b2, key_tensors=(f.w1, f.b1, f.w2, f.b2))
    opts = ops.RenderOptions(samples=int(depth_samples_per_ray), fine=bool(cfg.fine_sampling),
                             white_background=bool(cfg.white_background), randomize=bool(randomize),
                             scene_range=float(cfg.scene_range), inv_alpha=1.0 / float(f.alpha),
                             beta=float(f.beta), extras=extras, heads=heads)
    out = ops.volume_render(planes_tm, palette, ro, rd, near, far, dec, opts,
                            u_coarse=u_coarse, u_fine=u_fine, seed=seed, debug=debug, xray=xray, vhead=vhead)
    if extras:
        rgb, depth, mask, normals, semantics = out
        if semantics is not None and extras & 2 and 0 < f.attention_values < MAX_ATTENTION:
            semantics = semantics[..., :int(f.attention_values)]
    else:
        (rgb, depth, mask), normals, semantics = out, None, None
    if depth_mode == 'zbuffer':
        depth = zbuffer_depth(depth, rd, tform_cam2world)
    return rgb, depth, mask, normals, semantics, dict(f.model_outputs)


def zbuffer_depth(depth, ray_directions, tform_cam2world):
    """eval_{nusc,kitti,waymo}_persp.py:221-228: the compositing depth (a
    distance along the unit ray) -> camera-space z of the flipped camera,
    -(R_world2cam · rd)_z · depth.  No gradient: the depth map carries none (nerf_utils.py:151)
    and the eval scripts' losses never read it."""
    from .inversion import invert_space
    with torch.no_grad():
        w2c = invert_space(tform_cam2world.detach())
        view = torch.sum(ray_directions.detach()[..., None, :] * w2c[:, None, None, :3, :3], dim=-1)
        return (view * depth.unsqueeze(-1))[..., -1] * (-1)


def render_zbuffer(*args, **kwargs):
    """The render() copy of the perspective eval scripts (eval_nusc_persp.py:43-231,
    eval_kitti_persp.py, eval_waymo_persp.py): run.py's render with the depth map converted to
    camera-space z (zbuffer_depth).  Same signature as render."""
    return render(*args, depth_mode='zbuffer', **kwargs)
