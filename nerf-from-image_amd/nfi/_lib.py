"""ctypes binding of the nfi C-ABI (include/nfi.h) — the binding a reference-side maintainer
would add.  Loads the in-tree HIP library `libnfi_hip.so`; there is no
fallback: if the library is missing or was built for another ABI, importing the renderer
raises.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('NFI_LIBRARY') or os.path.join(_HERE, 'libnfi_hip.so')
ABI_VERSION = 18
DEC_SIZE = 7200
DEC_SIZE_VIEWDIR = 14384

c_float_p = ctypes.POINTER(ctypes.c_float)
c_void_p = ctypes.c_void_p


class NfiCamera(ctypes.Structure):
    _fields_ = [('cam', c_void_p), ('focal', c_void_p), ('center', c_void_p), ('bbox', c_void_p),
                ('B', ctypes.c_int32), ('H', ctypes.c_int32), ('W', ctypes.c_int32),
                ('_pad', ctypes.c_int32)]


class NfiField(ctypes.Structure):
    _fields_ = [('planes', c_void_p), ('sb', ctypes.c_int64), ('sq', ctypes.c_int64),
                ('st', ctypes.c_int64), ('R', ctypes.c_int32), ('_pad', ctypes.c_int32),
                ('dec', c_void_p), ('palette', c_void_p), ('inv_alpha', ctypes.c_float),
                ('beta', ctypes.c_float), ('scene_range', ctypes.c_float),
                ('heads', ctypes.c_int32), ('xray', c_void_p), ('vhead', c_void_p),
                ('vhead_out', ctypes.c_int32), ('_pad2', ctypes.c_int32)]


class NfiRenderArgs(ctypes.Structure):
    _fields_ = [('field', NfiField), ('ro', c_void_p), ('rd', c_void_p), ('near_', c_void_p),
                ('far_', c_void_p), ('B', ctypes.c_int32), ('HW', ctypes.c_int32),
                ('S', ctypes.c_int32), ('fine', ctypes.c_int32), ('white_bg', ctypes.c_int32),
                ('randomize', ctypes.c_int32), ('W', ctypes.c_int32), ('_pad3', ctypes.c_int32),
                ('seed', ctypes.c_uint64),
                ('offset', ctypes.c_uint64), ('u_coarse', c_void_p), ('u_fine', c_void_p),
                ('rgb', c_void_p), ('depth', c_void_p), ('mask', c_void_p),
                ('t_saved', c_void_p), ('sigma_saved', c_void_p), ('rgb_saved', c_void_p),
                ('y_saved', c_void_p), ('perm', c_void_p), ('x_saved', c_void_p),
                ('tile_counts', c_void_p), ('extras', ctypes.c_int32), ('_pad4', ctypes.c_int32),
                ('normal_map', c_void_p), ('semantic_map', c_void_p),
                ('z_coarse', c_void_p), ('z_fine', c_void_p)]


class NfiRenderGradArgs(ctypes.Structure):
    _fields_ = [('g_rgb', c_void_p), ('g_mask', c_void_p), ('d_planes', c_void_p),
                ('d_palette_ray', c_void_p), ('g_ro', c_void_p), ('g_rd', c_void_p),
                ('tile_counts', c_void_p), ('workspace', c_void_p), ('workspace_bytes', ctypes.c_int64),
                ('d_xray', c_void_p)]


# symbol -> (restype, argtypes); every entry point of include/nfi.h
SIGNATURES = {
    'nfi_abi_version': (ctypes.c_int32, []),
    'nfi_last_error': (ctypes.c_char_p, []),
    'nfi_decoder_pack': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, c_void_p, c_void_p]),
    'nfi_decoder_size': (ctypes.c_int64, [ctypes.c_int32]),
    'nfi_decoder_pack_n': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                            ctypes.c_float, ctypes.c_float, ctypes.c_float, c_void_p, c_void_p]),
    'nfi_planes_to_texel_major': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                   c_void_p, c_void_p]),
    'nfi_planes_to_channel_major': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                     c_void_p, c_void_p]),
    'nfi_set_deterministic': (ctypes.c_int32, [ctypes.c_int32]),
    'nfi_pose_forward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int32] * 2 + [c_void_p] * 3),
    'nfi_pose_backward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int32] * 2 + [c_void_p] * 7),
    'nfi_pose_project': (ctypes.c_int32, [c_void_p] * 3 + [ctypes.c_int32, c_void_p]),
    'nfi_rays_forward': (ctypes.c_int32, [ctypes.POINTER(NfiCamera), ctypes.c_float, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'nfi_rays_backward': (ctypes.c_int32, [ctypes.POINTER(NfiCamera), c_void_p, c_void_p,
                                           c_void_p, c_void_p]),
    'nfi_segment_sum': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         c_void_p, c_void_p, c_void_p]),
    'nfi_render_forward': (ctypes.c_int32, [ctypes.POINTER(NfiRenderArgs), c_void_p]),
    'nfi_render_backward_workspace_bytes': (ctypes.c_int64, [ctypes.POINTER(NfiRenderArgs)]),
    'nfi_tile_count_size': (ctypes.c_int64, [ctypes.POINTER(NfiRenderArgs)]),
    'nfi_tile_count_size_shape': (ctypes.c_int64, [ctypes.c_int32] * 5),
    'nfi_render_backward': (ctypes.c_int32, [ctypes.POINTER(NfiRenderArgs),
                                             ctypes.POINTER(NfiRenderGradArgs), c_void_p]),
    'nfi_render_backward_stage': (ctypes.c_int32, [ctypes.POINTER(NfiRenderArgs),
                                                   ctypes.POINTER(NfiRenderGradArgs), ctypes.c_int32,
                                                   c_void_p]),
    # per-stage seams (include/nfi.h, ABI 12)
    'nfi_near_far_workspace_bytes': (ctypes.c_int64, [ctypes.c_int64]),
    'nfi_near_far': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_float, c_void_p, c_void_p,
                                      c_void_p, c_void_p]),
    'nfi_sample_pdf': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_void_p,
                                        c_void_p]),
    'nfi_composite_forward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
                              + [c_void_p] * 5),
    'nfi_composite_backward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
                               + [c_void_p] * 8),
    'nfi_sampler_chunks': (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int64]),
    'nfi_sampler_forward': (ctypes.c_int32, [ctypes.POINTER(NfiField), c_void_p, ctypes.c_int32, ctypes.c_int64,
                                             c_void_p, c_void_p, c_void_p, c_void_p]),
    'nfi_sampler_backward': (ctypes.c_int32, [ctypes.POINTER(NfiField), c_void_p, ctypes.c_int32, ctypes.c_int64]
                             + [c_void_p] * 7),
    # the remaining nerf_utils seams (ABI 15)
    'nfi_ray_bundle': (ctypes.c_int32, [ctypes.POINTER(NfiCamera), c_void_p, c_void_p, c_void_p]),
    'nfi_ray_bundle_backward': (ctypes.c_int32, [ctypes.POINTER(NfiCamera), c_void_p, c_void_p, c_void_p,
                                                 c_void_p]),
    'nfi_query_points': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, c_void_p,
                                                          ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p,
                                                          c_void_p]),
    'nfi_query_points_backward': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int32, c_void_p,
                                                   c_void_p, c_void_p]),
    'nfi_cumprod_exclusive': (ctypes.c_int32, [c_void_p, ctypes.c_int64, ctypes.c_int32, c_void_p, c_void_p]),
    'nfi_cumprod_exclusive_backward': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int32,
                                                        c_void_p, c_void_p]),
    'nfi_volume_weights_forward': (ctypes.c_int32, [c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int32, c_void_p,
                                                                     c_void_p]),
    'nfi_volume_weights_backward': (ctypes.c_int32, [c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int32]
                                    + [c_void_p] * 5),
    # include/nfi_producer.h
    'nfi_split16_pack': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int64, c_void_p, c_void_p, c_void_p,
                                          c_void_p]),
    'nfi_wino_input_transform_max': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_split16_slot_words': (ctypes.c_int32, []),
    'nfi_absmax_slots': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int64, c_void_p, c_void_p]),
    'nfi_gemm_split16': (ctypes.c_int32, [c_void_p] * 6 + [ctypes.c_int32] * 5 + [c_void_p]),
    'nfi_gemm_split16_shared_a': (ctypes.c_int32, [c_void_p] * 6 + [ctypes.c_int32] * 5 + [c_void_p] * 2),
    'nfi_gemm_split16_ksplit': (ctypes.c_int32, [c_void_p] * 6 + [ctypes.c_int32] * 6 + [c_void_p] * 2),
    'nfi_syn_cond_norm_act_forward': (ctypes.c_int32, [c_void_p] * 3 + [ctypes.c_int32] * 3 + [c_void_p] * 3),
    'nfi_syn_cond_norm_act_backward': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 3 + [c_void_p] * 4),
    'nfi_syn_act_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_float, c_void_p]),
    'nfi_syn_act_backward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_float, c_void_p]),
    'nfi_syn_fir_up_act_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                    ctypes.c_float, c_void_p]),
    'nfi_syn_fir_up_backward': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                 c_void_p]),
    'nfi_syn_up_conv_scatter': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, c_void_p]),
    'nfi_syn_up_conv_gather': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_int32, c_void_p]),
    'nfi_syn_up_conv_act_backward': (ctypes.c_int32, [c_void_p] * 6 + [ctypes.c_int32] * 3
                                     + [ctypes.c_float, c_void_p]),
    'nfi_syn_up_conv_act_backward_max': (ctypes.c_int32, [c_void_p] * 7 + [ctypes.c_int32] * 3
                                         + [ctypes.c_float, c_void_p]),
    'nfi_syn_up_conv_fir_act_forward': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 3
                                        + [ctypes.c_float, c_void_p]),
    'nfi_aug_sample_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p] + [ctypes.c_int32] * 6
                               + [ctypes.c_float, c_void_p]),
    'nfi_aug_sample_backward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p] + [ctypes.c_int32] * 6
                                + [c_void_p]),
    'nfi_aug_affine_grid': (ctypes.c_int32, [c_void_p] + [ctypes.c_int32] * 3 + [c_void_p, c_void_p]),
    'nfi_syn_up_add_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_vgg_first_forward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_vgg_first_forward_max': (ctypes.c_int32, [c_void_p] * 7 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_vgg_first_backward_scaled': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_vgg_first_backward': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_syn_up_add_forward_strided': (ctypes.c_int32, [c_void_p] * 7 + [ctypes.c_int32] * 3 + [c_void_p]),
    'nfi_syn_up_backward_strided': (ctypes.c_int32, [c_void_p] * 4 + [ctypes.c_int32] * 3 + [c_void_p]),
    'nfi_syn_up_backward': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                             c_void_p]),
    'nfi_syn_scale_backward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_lpips_head_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_int32, c_void_p]),
    'nfi_lpips_head_backward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, c_void_p]),
    'nfi_vgg_bias_relu_forward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p,
                                                   ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_int32, c_void_p]),
    'nfi_vgg_relu_backward_max': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_vgg_relu_backward': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_wino_weight_transform': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_int32, c_void_p]),
    'nfi_wino_input_transform': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                  ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_wino_input_transform_scaled': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_wino_output_transform': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                                   ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_wino_packed_size': (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    'nfi_wino_conv_fused_split': (ctypes.c_int32, [c_void_p] * 7 + [ctypes.c_int32] * 5 + [c_void_p]),
    'nfi_wino_input_transform_relu_grad': (ctypes.c_int32, [c_void_p] * 3 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_wino_output_transform_scaled_grad': (ctypes.c_int32, [c_void_p] * 5 + [ctypes.c_int32] * 4 + [c_void_p]),
    'nfi_wino_pack_weights': (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32, ctypes.c_int32, c_void_p]),
    'nfi_wino_conv_fused': (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             c_void_p]),
    'nfi_dconv_pack': (ctypes.c_int32, [c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_void_p, c_void_p,
                                        c_void_p]),
    'nfi_dconv3x3': (ctypes.c_int32, [c_void_p] * 10 + [ctypes.c_int32] * 5 + [c_void_p]),
    'nfi_absmax_scaled_slots': (ctypes.c_int32, [c_void_p, c_void_p] + [ctypes.c_int32] * 3 + [c_void_p, c_void_p]),
}

_lib = None
_lock = threading.Lock()


class NfiError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load and type the library once.  Raises NfiError if it is absent or mismatched."""
    global _lib
    if _lib is not None:     # (fast path: every launch goes through here)
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NfiError(f'nfi HIP library not found at {path}; build it with '
                           f'`python __graft_entry__.py` (build()) — there is no CPU fallback')
        lib = ctypes.CDLL(path)
        # NFI_AB_OLDER=1 (A/B timing of an older build through scripts/ab_multi.sh only): entry points
        # the older library lacks stay unbound and an older ABI version is accepted (the render
        # structs are unchanged since ABI 14); never set for product runs
        ab_older = (os.environ.get('NFI_AB_OLDER') == '1'
                    and os.path.abspath(path) != os.path.join(_HERE, 'libnfi_hip.so'))
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                if ab_older:
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        v = lib.nfi_abi_version()
        if v != ABI_VERSION and not (ab_older and v >= 14):
            raise NfiError(f'nfi ABI mismatch: library {v}, binding {ABI_VERSION}')
        _lib = lib
        return lib


def check(code: int, what: str):
    if code != 0:
        msg = _lib.nfi_last_error().decode() if _lib is not None else ''
        raise NfiError(f'{what} failed ({code}): {msg}')
