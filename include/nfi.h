/*
 * nfi.h — C-ABI of the MI355X-native volume renderer for the SDF-NeRF inversion loop of
 * yuliangguo/nerf-from-image (reference @ 2024-10-08).
 *
 * The reference has no FFI: its renderer is plain Python/PyTorch.  The seams this library
 * replaces are:
 *   render()                                run.py:176-350
 *   nerf_utils.get_ray_bundle               lib/nerf_utils.py:28-93
 *   nerf_utils.compute_near_far_planes      lib/nerf_utils.py:227-275
 *   nerf_utils.compute_query_points_from_rays  lib/nerf_utils.py:96-122
 *   Generator.forward's `sampler` closure   models/generator.py:587-681
 *   TriplanarDecoder.forward                models/generator.py:301-331
 *   nerf_utils.render_volume_density_weights_only + EG3D smoothing  nerf_utils.py:166-182, run.py:261-272
 *   nerf_utils.sample_pdf                   lib/nerf_utils.py:185-224
 *   sort/merge of coarse+fine samples       run.py:283-288, 312-319
 *   nerf_utils.render_volume_density        lib/nerf_utils.py:125-163
 * and their autograd backward passes.  INTEGRATION.md shows the ctypes binding the
 * reference side would add (nerf-from-image_amd/nfi/_lib.py is that binding).
 *
 * Conventions: all pointers are DEVICE pointers to fp32 (unless stated), contiguous in the
 * layout given; `stream` is a hipStream_t (NULL = default stream).  Functions are
 * asynchronous on `stream`, allocate nothing, keep no state, and are safe to call from
 * several host threads on different streams/devices.  Return 0 on success, a negative
 * code on a bad argument (nothing launched) or a HIP launch failure; nfi_last_error()
 * returns a thread-local message.
 */
#ifndef NFI_H
#define NFI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFI_ABI_VERSION 18
#define NFI_DEC_SIZE 7200   /* floats in the packed decoder buffer (11 outputs: split-f16 tables) */
#define NFI_DEC_SIZE_VIEWDIR 14384 /* ... with the view-direction mapper (33 outputs) */

enum {
  NFI_OK = 0,
  NFI_EINVAL = -1,   /* bad argument / unsupported configuration */
  NFI_ELAUNCH = -2,  /* HIP launch error */
  NFI_ECHECK = -3,   /* integrity check of an -DNFI_TILE_CHECK debug build failed (never in the product) */
};

/* Camera batch (nerf_utils.py:28-93): cam2world [B,4,4]; focal [B] (NULL = orthographic
 * projection, nerf_utils.py:67-91); optional center [B,2] (:43-47) and bbox [B,2,2] (:52-56). */
typedef struct nfi_camera {
  const float* cam;
  const float* focal;
  const float* center;
  const float* bbox;
  int32_t B, H, W;
  int32_t _pad;
} nfi_camera;

/* Radiance field (generator.py:288-331, 587-681; stylegan.py:148-180).
 * planes: texel-major tri-planes; element (b, plane q, row y, col x, channel c) lives at
 *   planes[b*sb + q*sq + (y*R + x)*st + c]   (c contiguous; 32 channels; q = xy, xz, yz).
 * dec: packed, gain-scaled decoder from nfi_decoder_pack().
 * palette: attention values [B,10,3] (AttentionMapper output, generator.py:455-462).
 * inv_alpha = 1/Generator.alpha, beta = Generator.beta (generator.py:397-399, 629-636).
 * heads: the reference's field variants (sampler closure, generator.py:628-679), 0 = the
 *   inversion field (SDF density, attention colour) or an OR of
 *   NFI_HEAD_RGB_SIGMOID   --attention_values 0: rgb = wide_sigmoid_rescaled(features[0..2])
 *                          (:665-666, :36-39); decoder [4,64] zero-padded to [11,64]; palette
 *                          unused (may be NULL); no semantics
 *   NFI_HEAD_NERF_DENSITY  use_sdf False: sigma = softplus(d - 1) * (1 - mask) (:637-641);
 *                          inv_alpha / beta unused; no normals
 *   NFI_HEAD_VIEWDIR       --use_viewdir (generator.py:189-252, 376-377, 661-663): the decoder has
 *                          33 outputs (distance + 32 features; dec packed with nout 33) and the
 *                          colour logits are output(leaky_relu(xray + features, 0.2)) with
 *                          xray [B*HW,32] the per-ray mapper trunk of the ray direction
 *                          (ViewDirectionMapper.forward :223-238, computed by the caller) and
 *                          vhead the gain-scaled output layer: [vhead_out,32] weights then
 *                          [vhead_out] bias, vhead_out = 10 (attention) or 3 (RGB_SIGMOID) */
#define NFI_HEAD_RGB_SIGMOID 1
#define NFI_HEAD_NERF_DENSITY 2
#define NFI_HEAD_VIEWDIR 4
typedef struct nfi_field {
  const float* planes;
  int64_t sb, sq, st;
  int32_t R;
  int32_t _pad;
  const float* dec;
  const float* palette;
  float inv_alpha, beta, scene_range;
  int32_t heads;
  const float* xray;   /* NFI_HEAD_VIEWDIR only (else NULL) */
  const float* vhead;
  int32_t vhead_out;
  int32_t _pad2;
} nfi_field;

/* One render call: rays of B images × HW pixels, S coarse samples (+ S fine if fine). */
typedef struct nfi_render_args {
  nfi_field field;
  const float* ro;     /* [B*HW,3] ray origins */
  const float* rd;     /* [B*HW,3] unit ray directions (after F.normalize, run.py:196) */
  const float* near_;  /* [B*HW] */
  const float* far_;   /* [B*HW] */
  int32_t B, HW, S;
  int32_t fine;        /* args.fine_sampling (run.py:259) */
  int32_t white_bg;    /* dataset_config['white_background'] */
  int32_t randomize;   /* stratified jitter + random u in sample_pdf (else linspace) */
  int32_t W;           /* image width (HW = H*W): with H, W multiples of 16 the kernels walk rays in
                          16x16-pixel tiles dealt round-robin over the XCDs (L2 locality); 0 = off */
  int32_t _pad3;
  uint64_t seed, offset;       /* Philox stream when u_* are NULL */
  const float* u_coarse;       /* optional [B*HW,S] injected jitter (nerf_utils.py:120) */
  const float* u_fine;         /* optional [B*HW,S] injected u (nerf_utils.py:202-205) */
  /* forward outputs */
  float* rgb;          /* [B*HW,3] */
  float* depth;        /* [B*HW]   */
  float* mask;         /* [B*HW]   */
  /* per-ray state kept for backward: merged, sorted samples (N = fine ? 2S : S).  t/sigma/rgb/y/perm
     are all set or all NULL: NULL = a forward-only call (no backward, extras or tile counts) */
  float* t_saved;      /* [B*HW,N]   */
  float* sigma_saved;  /* [B*HW,N]   */
  float* rgb_saved;    /* [B*HW,3,N] */
  float* y_saved;      /* [B*HW,NOUT,N] decoder outputs (distance, 10 logits; NOUT = 33 with
                          NFI_HEAD_VIEWDIR: distance, 32 features) in evaluation order:
                          coarse 0..S-1 then fine S..2S-1 (lets the backward skip the forward MLP) */
  int16_t* perm;       /* [B*HW,N] merged sample k -> evaluation index */
  float* x_saved;      /* [B*HW*N,32] decoder inputs (mean tap features) in evaluation order; optional
                          in the forward (NULL: not written), required by the backward */
  int32_t* tile_counts; /* optional [nfi_tile_count_size()] per-plane-tile sample counts for the
                           backward's d-planes binning (zeroed and filled by the forward); NULL = skip */
  int32_t extras;      /* eval outputs (run.py:227-257, 293-335): bit 1 normals, 2 semantics, 4 coords
                          (the coords map replaces the semantic map, run.py:334-335).  Need y_saved
                          and perm, normals also x_saved; the maps carry no gradient (their callers
                          are eval renders, run.py:1250-1264) */
  int32_t _pad4;
  float* normal_map;   /* [B*HW,3]  (extras & 1): sum_i w_i normalize(d sdf_i / d p_i) (+1-mask if white) */
  float* semantic_map; /* [B*HW,10] (extras & 2: sum_i w_i softmax_i) or [B*HW,3] (extras & 4: sum_i w_i p_i) */
  float* z_coarse;     /* optional [B*HW,S] debug: coarse depths */
  float* z_fine;       /* optional [B*HW,S] debug: fine depths, sorted */
} nfi_render_args;

typedef struct nfi_render_grad_args {
  const float* g_rgb;   /* [B*HW,3] dL/d rgb  */
  const float* g_mask;  /* [B*HW]   dL/d mask (depth carries no gradient, nerf_utils.py:151) */
  float* d_planes;      /* same layout/strides as field.planes; ACCUMULATED into (zero it) */
  float* d_palette_ray; /* [B*HW*ceil(N/64),30] per-(ray, 64-sample chunk) partial dL/d palette
                           (reduce per image with nfi_segment_sum, M = HW*ceil(N/64)) */
  float* g_ro;          /* [B*HW,3] dL/d ray origins  (NULL: skip coordinate gradients) */
  float* g_rd;          /* [B*HW,3] dL/d unit ray directions */
  const int32_t* tile_counts; /* the forward's tile_counts, or NULL (the backward counts itself) */
  void* workspace;      /* device scratch of nfi_render_backward_workspace_bytes() bytes */
  int64_t workspace_bytes;
  float* d_xray;        /* NFI_HEAD_VIEWDIR: [B*HW*ceil(N/64),32] per-(ray, 64-sample chunk) partial dL/d xray
                           (written; the caller sums each ray's chunks); else NULL */
} nfi_render_grad_args;

int32_t nfi_abi_version(void);
const char* nfi_last_error(void);

/* EqualizedLinear parameters (stylegan.py:173-176) -> packed, gain-scaled decoder:
 * W1s = w1*g1 [64,32], b1s = b1*gb, W2s = w2*g2 [11,64], b2s = b2*gb (a [4,64] decoder of
 * NFI_HEAD_RGB_SIGMOID is passed zero-padded to 11 rows).  The 11-output decoder is packed for
 * the f16 matrix cores: every weight times a per-matrix power of two as an fp16 pair hi + lo
 * (fp32-accurate three-product contractions; NFI_DEC_SIZE floats, one workgroup launch). */
int32_t nfi_decoder_pack(const float* w1, const float* b1, const float* w2, const float* b2,
                         float g1, float g2, float gb, float* dec, void* stream);
/* The same for a decoder of nout outputs: 11 (= nfi_decoder_pack) or 33 (NFI_HEAD_VIEWDIR:
 * TriplanarDecoder(32, 32), generator.py:376-377); w2 [nout,64], b2 [nout]; dec holds
 * nfi_decoder_size(nout) floats. */
int64_t nfi_decoder_size(int32_t nout);
int32_t nfi_decoder_pack_n(const float* w1, const float* b1, const float* w2, const float* b2, int32_t nout,
                           float g1, float g2, float gb, float* dec, void* stream);

/* [B,3,32,R,R] channel-major planes (generator.py:476-477) <-> texel-major [B,3,R,R,32]. */
int32_t nfi_planes_to_texel_major(const float* src, int32_t B, int32_t R, float* dst, void* stream);
int32_t nfi_planes_to_channel_major(const float* src, int32_t B, int32_t R, float* dst, void* stream);
/* The inversion step's pose algebra (run.py:2262: pose_to_matrix(z0, t2, s, F.normalize(q)),
 * lib/pose_utils.py:48-78) and its backward, one launch each; [B] z0 (NULL: no focal, orthographic
 * branch), [B,2] t2, [B] s, [B,4] q (w, x, y, z; normalised inside) -> cam2world [B,4,4], focal [B]
 * (= (1 + exp z0) / 2).  The backward writes (not accumulates) d z0 / d t2 / d s / d q from
 * d cam2world and d focal (NULL: zero).  nfi_pose_project: the post-step projections in place
 * (run.py:2300-2306): q <- F.normalize(q), z0 <- clamp(z0, -4, 4), s <- |s| (z0 / s may be NULL). */
int32_t nfi_pose_forward(const float* z0, const float* t2, const float* s, const float* q, int32_t B,
                         int32_t camera_flipped, float* cam2world, float* focal, void* stream);
int32_t nfi_pose_backward(const float* z0, const float* t2, const float* s, const float* q, int32_t B,
                          int32_t camera_flipped, const float* g_cam2world, const float* g_focal, float* d_z0,
                          float* d_t2, float* d_s, float* d_q, void* stream);
int32_t nfi_pose_project(float* z0, float* s, float* q, int32_t B, void* stream);

/* get_ray_bundle + F.normalize + compute_near_far_planes (run.py:193-200).
 * Outputs ro, rd (unit) [B*H*W,3], near, far [B*H*W].  ws: 2 + B*H*W uint32 of device scratch. */
int32_t nfi_rays_forward(const nfi_camera* cam, float scene_range, float* ro, float* rd,
                         float* near_, float* far_, uint32_t* ws, void* stream);

/* Backward of get_ray_bundle + F.normalize: g_ro, g_rd [B*H*W,3] -> per-pixel partials
 * contrib [B*H*W,16] = {d cam[0..2][0..3] (12), d cam[3][3], d focal, 0, 0}. */
int32_t nfi_rays_backward(const nfi_camera* cam, const float* g_ro, const float* g_rd,
                          float* contrib, void* stream);

/* out[b,k] = sum_m in[b,m,k]  (deterministic two-pass); ws >= B*64*K floats. */
int32_t nfi_segment_sum(const float* in, int32_t B, int32_t M, int32_t K, float* out, float* ws,
                        void* stream);

/* Fused forward: stratified samples -> field -> coarse weights + EG3D smoothing -> sample_pdf
 * -> fine samples -> field -> sort/merge -> compositing.  Supported S: 3..128 with fine
 * sampling (N = 2S merged samples), 1..256 without. */
int32_t nfi_render_forward(const nfi_render_args* a, void* stream);

/* Backward of nfi_render_forward from its saved state: per-ray compositing backward, then the
 * field backward (decoder input-gradient on the saved decoder inputs) writes per-sample feature
 * gradients and appends each (sample, plane) entry to its 7x4-cell plane tile's bin; d planes is
 * summed per tile chunk in registers and flushed once per chunk, each entry's grid gradient
 * computed there against the tile's texels; d ray origins / directions are reduced per ray. */
int64_t nfi_render_backward_workspace_bytes(const nfi_render_args* a);
int64_t nfi_tile_count_size(const nfi_render_args* a);   /* = B * beams * 3 * ((R-2)/7+1) * ((R-2)/4+1),
                                                            beams = 1 unless built with NFI_BEAM_SAMPLES */
/* The same size from the shapes alone (B images of H x W rays, N samples per ray, planes R x R): for
 * shape-only callers (the TORCH_LIBRARY Meta kernels) that hold no argument block; -1 on bad shapes. */
int64_t nfi_tile_count_size_shape(int32_t B, int32_t R, int32_t H, int32_t W, int32_t N);
/* Deterministic backward for the calling host thread (on = 1), the default atomics form (0), or
 * query only (-1); returns the previous setting (initially from the environment variable
 * NFI_DETERMINISTIC).  The setting is PER HOST THREAD and is read by the thread that calls
 * nfi_render_backward[_stage] / nfi_render_backward_workspace_bytes: a caller that sets it on one
 * thread does not change a backward another thread runs (PyTorch autograd runs .backward() on its
 * device thread; nfi.ops sets it there from nfi.ops.DETERMINISTIC / torch.use_deterministic_algorithms
 * around each backward and restores that thread's previous value).  Deterministic: every tile's bin entries are sorted by sample index before the
 * tile pass and the d planes are summed from per-chunk partial tile images in a fixed order instead
 * of float atomics, so d planes (and every other output) are bitwise reproducible run to run; the
 * workspace (nfi_render_backward_workspace_bytes, which follows this setting) grows by ~40 B per
 * (sample, plane) entry.  The reference's grid_sample backward itself accumulates with atomics. */
int32_t nfi_set_deterministic(int32_t on);
int32_t nfi_render_backward(const nfi_render_args* a, const nfi_render_grad_args* g, void* stream);
/* The same backward one stage at a time, in order 0, 1, 2 on one stream with one workspace
 * (lets a caller time or overlap the stages): 0 = tile binning of the saved samples,
 * 1 = compositing + field backward (d palette, per-sample feature gradients, tile entries),
 * 2 = per-tile d planes accumulation + grid gradients, then d rays. */
int32_t nfi_render_backward_stage(const nfi_render_args* a, const nfi_render_grad_args* g, int32_t stage,
                                  void* stream);

/* ---- Per-stage seams: the reference's nerf_utils functions and the sampler
 * closure as launches of their own, for a caller that uses one of them without render().
 * Same conventions (device pointers, caller's stream, no allocation). */

/* compute_near_far_planes (lib/nerf_utils.py:227-275) on n rays ro, rd [n,3] (directions taken as
 * given): slab test against [-scene_range, scene_range]^3; rays that miss get the min near / max far
 * of the hits of the call (:260-261); near, far clamped to >= 0.1, far >= near + 1e-3 (:264-270).
 * ws: nfi_near_far_workspace_bytes(n) bytes of device scratch.  No ray hitting the box: the
 * reference raises (min() of an empty tensor); here near = 0.1, far = 0.101. */
int64_t nfi_near_far_workspace_bytes(int64_t n);
int32_t nfi_near_far(const float* ro, const float* rd, int64_t n, float scene_range, float* near_, float* far_,
                     void* ws, void* stream);

/* sample_pdf (lib/nerf_utils.py:185-224): bins [n,nbins], weights [n,nbins-1] -> out [n,num_samples]
 * (2 <= nbins <= 1024).  deterministic: u = linspace(0, 1, num_samples); else u [n,num_samples] if
 * given (the reference's torch.rand draws), or a Philox-4x32-10 stream of (seed, offset).  No
 * gradient (the reference samples under no_grad, run.py:259-281). */
int32_t nfi_sample_pdf(const float* bins, const float* weights, int64_t n, int32_t nbins, int32_t num_samples,
                       int32_t deterministic, const float* u, uint64_t seed, uint64_t offset, float* out,
                       void* stream);

/* get_ray_bundle (lib/nerf_utils.py:28-93) alone: ro, rd [B*H*W,3], rd NOT normalised (render() runs
 * F.normalize after it, run.py:196; nfi_rays_forward fuses both).  Backward: g_ro, g_rd of these raw
 * directions -> per-pixel partials contrib [B*H*W,16] in nfi_rays_backward's layout (d cam 12, d cam[3][3],
 * d focal); no gradient to center / bbox (dataset inputs in the reference). */
int32_t nfi_ray_bundle(const nfi_camera* cam, float* ro, float* rd, void* stream);
int32_t nfi_ray_bundle_backward(const nfi_camera* cam, const float* g_ro, const float* g_rd, float* contrib,
                                void* stream);

/* compute_query_points_from_rays (lib/nerf_utils.py:96-122) on n rays ro, rd [n,3], near, far [n]:
 * depth [n,S] = lerp(near, far, i/S) (+ u (far - near)/S if randomize: u [n,S] given, or the Philox
 * stream of (seed, offset) the fused render draws its coarse jitter from), points [n,S,3] = ro + rd t.
 * Backward (to the rays; the depth values carry none, near/far being detached, run.py:197-200):
 * g_points [n,S,3] -> d_ro, d_rd [n,3] (either may be NULL). */
int32_t nfi_query_points(const float* ro, const float* rd, const float* near_, const float* far_, int64_t n,
                         int32_t S, int32_t randomize, const float* u, uint64_t seed, uint64_t offset, float* points,
                         float* depth, void* stream);
int32_t nfi_query_points_backward(const float* depth, const float* g_points, int64_t n, int32_t S, float* d_ro,
                                  float* d_rd, void* stream);

/* cumprod_exclusive (lib/nerf_utils.py:20-25) along the last axis of x [n,N]: out[:,0] = 1,
 * out[:,k] = prod_{j<k} x[:,j] (product carried in fp64, as ATen's CPU cumprod of float).
 * Backward: g_out [n,N] -> d_x [n,N] (no division: exact zeros handled; d_x[:,N-1] = 0; N <= 1024). */
int32_t nfi_cumprod_exclusive(const float* x, int64_t n, int32_t N, float* out, void* stream);
int32_t nfi_cumprod_exclusive_backward(const float* x, const float* g_out, int64_t n, int32_t N, float* d_x,
                                       void* stream);

/* render_volume_density_weights_only (lib/nerf_utils.py:166-182): sigma [n,N], rd [n,3], t [n,N] ->
 * weights [n,N] (1 <= N <= 1024).  Backward: dL/d weights -> d sigma [n,N] (written), d rd [n,3] and
 * d t [n,N] (optional). */
int32_t nfi_volume_weights_forward(const float* sigma, const float* rd, const float* t, int64_t n, int32_t N,
                                   float* weights, void* stream);
int32_t nfi_volume_weights_backward(const float* sigma, const float* rd, const float* t, int64_t n, int32_t N,
                                    const float* g_weights, float* d_sigma, float* d_rd, float* d_t, void* stream);

/* render_volume_density (lib/nerf_utils.py:125-163, with cumprod_exclusive :20-25) on n rays of
 * N samples (1 <= N <= 1024): sigma [n,N], rgb [n,N,3], rd [n,3] (distances are scaled by ||rd||),
 * t [n,N] depth values -> rgb_map [n,3] (+ 1 - mask if white_bg), depth [n] (detached weights),
 * mask [n], and the weights [n,N] if `weights` is not NULL (for the normal / semantic maps a caller
 * builds on them, :150-157).  Backward: dL/d rgb_map, dL/d mask and optionally dL/d weights
 * [n,N] -> d sigma [n,N], d rgb [n,N,3] (written), d rd [n,3] and d t [n,N] (each optional). */
int32_t nfi_composite_forward(const float* sigma, const float* rgb, const float* rd, const float* t, int64_t n,
                              int32_t N, int32_t white_bg, float* rgb_map, float* depth, float* mask, float* weights,
                              void* stream);
int32_t nfi_composite_backward(const float* sigma, const float* rgb, const float* rd, const float* t, int64_t n,
                               int32_t N, int32_t white_bg, const float* g_rgb, const float* g_mask,
                               const float* g_weights, float* d_sigma, float* d_rgb, float* d_rd, float* d_t,
                               void* stream);

/* The sampler closure of Generator.forward (models/generator.py:587-681; TriplanarDecoder :301-331)
 * at caller points x [B,P,3] (world coordinates; image b's points read image b's planes and
 * palette): sigma [B*P], rgb [B*P,3] and, if y is not NULL, the decoder outputs y [B*P,11]
 * (distance + 10 logits, or + 3 colour features zero-padded with NFI_HEAD_RGB_SIGMOID) from which a
 * caller forms 'sdf_distance' / 'semantics'.  heads: 0, NFI_HEAD_RGB_SIGMOID, NFI_HEAD_NERF_DENSITY
 * (the view-direction closure needs per-ray inputs: render() only).
 * Backward: dL/d sigma, dL/d rgb, dL/d y (each optional) -> d planes (ACCUMULATED into, field.planes'
 * layout; NULL skips it), per-chunk dL/d palette partials d_palette_part [nfi_sampler_chunks(B,P),30] (reduce per
 * image with nfi_segment_sum, M = chunks / B; NULL with NFI_HEAD_RGB_SIGMOID) and d x [B*P,3]
 * (optional; grid_sampler_2d's border / align_corners grid gradient). */
int64_t nfi_sampler_chunks(int32_t B, int64_t P);
int32_t nfi_sampler_forward(const nfi_field* f, const float* x, int32_t B, int64_t P, float* sigma, float* rgb,
                            float* y, void* stream);
int32_t nfi_sampler_backward(const nfi_field* f, const float* x, int32_t B, int64_t P, const float* g_sigma,
                             const float* g_rgb, const float* g_y, float* d_planes, float* d_palette_part,
                             float* d_x, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NFI_H */
