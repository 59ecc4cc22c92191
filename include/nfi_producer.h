/*
 * nfi producer C-ABI: the memory-bound operators of the tri-plane producer (the StyleGAN2
 * synthesis network of yuliangguo/nerf-from-image, models/stylegan.py:293-490) around its
 * convolutions, fused for MI355X (gfx950), and the convolutions' own memory-bound halves: the
 * matrix products run as hipBLASLt GEMMs through PyTorch-ROCm (3x3: Winograd F(4,3), below;
 * up-sampling: one GEMM over the 9 taps + the tap scatter / gather here; 1x1: one batched GEMM
 * with the modulation folded into a per-image weight).  Everything between them is here:
 *
 *   modulated-conv epilogue  stylegan.py:140-145, 345-356   x*dcoefs + bias, *sqrt(2), leaky ReLU
 *   up-sampling FIR epilogue stylegan.py:99-103 (filter2d gain 4, pad 1) + the epilogue above
 *   skip-image upsample+add  stylegan.py:69-73, 428-433     upsample2d(img) + (toRGB conv + bias)
 *   channel-scale backward   stylegan.py:130                d(x*styles): g*styles and sum(g*x)
 *   LPIPS distance head      metrics.py:130-146 (lpips 0.1) normalise, difference, lin, mean
 *   LPIPS VGG16 epilogue     bias + ReLU (+ 2x2 max pool) after each trunk convolution
 *   LPIPS augmented copies   run.py:720-767 (grid_sample of 15 affine copies, gathered adjoint)
 *   LPIPS first layer        vgg16.features[0:2]: direct 3x3 conv + bias + ReLU, one pass each way
 *
 * Tensors are NCHW float32, contiguous; "planes" P = B*C images of one channel; per-plane
 * scales `d` have P entries ([B,C] row-major), per-channel biases C entries.  `stream` is a
 * hipStream_t.  Return NFI_OK (0) or a negative code (nfi_last_error() explains).  The
 * python-side mirror is nerf-from-image_amd/nfi/producer_ops.py.
 */
#ifndef NFI_PRODUCER_H
#define NFI_PRODUCER_H

#include <stdint.h>

#include "nfi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* y = lrelu(gain * (o * d[p] + bias[c]), 0.2) over P planes of HW (HW % 4 == 0).
 * Replaces stylegan.py:145 (x * dcoefs) + 348-356 (bias, act_gain, leaky_relu). */
int32_t nfi_syn_act_forward(const float* o, const float* d, const float* bias, float* y,
                            int32_t P, int32_t C, int32_t HW, float gain, void* stream);

/* Backward of nfi_syn_act_forward: gz = g * gain * slope(pre); go = gz * d[p];
 * dd[p] = sum_hw gz * o (dd is overwritten). */
int32_t nfi_syn_act_backward(const float* g, const float* o, const float* d, const float* bias,
                             float* go, float* dd, int32_t P, int32_t C, int32_t HW, float gain,
                             void* stream);

/* Up-sampling layer tail (stylegan.py:99-103 then the epilogue): t [P, 2n+1, 2n+1] (the stride-2
 * transposed-conv output) -> o = FIR_4x4(t) * 4 with pad 1 ([1,3,3,1] outer / 64), [P, 2n, 2n];
 * y = lrelu(gain * (o * d[p] + bias[c])).  o is written for the backward. */
int32_t nfi_syn_fir_up_act_forward(const float* t, const float* d, const float* bias, float* o,
                                   float* y, int32_t P, int32_t C, int32_t n, float gain,
                                   void* stream);

/* Adjoint of the 4x4 FIR (stylegan.py:36-46 EfficientResample backward): go [P,2n,2n] ->
 * gt [P,2n+1,2n+1]. */
int32_t nfi_syn_fir_up_backward(const float* go, float* gt, int32_t P, int32_t n, void* stream);

/* The stride-2 3x3 transposed convolution of the up-sampling layers (stylegan.py:99-101,
 * conv_transpose2d(x, w^T, stride=2)) as one GEMM over all 9 taps plus this scatter: the caller
 * computes P [B][9][C][n][n] = W9 x (W9 [9*C, Ci] = w permuted to [ky][kx][co][ci]); this sums the
 * taps into t [B][C][2n+1][2n+1], t[Y][X] = sum of P[3ky+kx][.][iy][ix] over Y = 2iy+ky, X = 2ix+kx. */
int32_t nfi_syn_up_conv_scatter(const float* P, float* t, int32_t B, int32_t C, int32_t n, void* stream);

/* The scatter fused with nfi_syn_fir_up_act_forward's FIR + epilogue (t stays on chip): P as
 * above -> o [B][C][2n][2n] (FIR output, for the backward) and y = lrelu(gain (o d[p] + bias[c])),
 * the operations of scatter then fir_up_act.  2n % 64 == 0. */
int32_t nfi_syn_up_conv_fir_act_forward(const float* P, const float* d, const float* bias, float* o, float* y,
                                        int32_t B, int32_t C, int32_t n, float gain, void* stream);

/* The backward of nfi_syn_up_conv_fir_act_forward's FIR + epilogue and of the scatter in one pass
 * (n % 32 == 0): g = d y [B][C][2n][2n], o (saved) -> dP [B][9][C][n][n] (the operand of the data
 * gradient W9^T dP) and dd[p] = sum gz o (overwritten) — nfi_syn_act_backward, then
 * nfi_syn_fir_up_backward, then nfi_syn_up_conv_gather, without go and gt in memory. */
int32_t nfi_syn_up_conv_act_backward(const float* g, const float* o, const float* d, const float* bias, float* dP,
                                     float* dd, int32_t B, int32_t C, int32_t n, float gain, void* stream);
/* The same, also leaving each image's running maximum of |dP| in its slots of vmax for the split-f16
 * product W9^T dP (nfi_gemm_split16_shared_a; vmax zero on entry, as nfi_wino_input_transform_max):
 * no separate maximum pass over dP. */
int32_t nfi_syn_up_conv_act_backward_max(const float* g, const float* o, const float* d, const float* bias, float* dP,
                                         float* dd, uint32_t* vmax, int32_t B, int32_t C, int32_t n, float gain,
                                         void* stream);

/* Its adjoint: gt [B][C][2n+1][2n+1] -> dP [B][9][C][n][n], dP[3ky+kx][c][iy][ix] =
 * gt[c][2iy+ky][2ix+kx]; the data gradient of the transposed convolution is then W9^T dP. */
int32_t nfi_syn_up_conv_gather(const float* gt, float* dP, int32_t B, int32_t C, int32_t n, void* stream);

/* Skip path (stylegan.py:428-433 + 380-381): out [P,2n,2n] = upsample2d(img [P,n,n]) + c +
 * bias[c]; img may be NULL (first block: out = c + bias). */
int32_t nfi_syn_up_add_forward(const float* img, const float* c, const float* bias, float* out,
                               int32_t P, int32_t C, int32_t n, void* stream);

/* Adjoint of upsample2d: g [P,2n,2n] -> gimg [P,n,n] (conv2d with the gain-4 FIR, stride 2,
 * pad 1; stylegan.py:79-83). */
int32_t nfi_syn_up_backward(const float* g, float* gimg, int32_t P, int32_t n, void* stream);

/* The skip path with channel-contiguous layouts: each tensor [B][C][h][w] is addressed by float
 * strides {b, q, t}: element (b, c, y, x) at b*sb + (c/32)*sq + (y*w + x)*st + c%32 — channels-last
 * [B][h][w][C] has sq = 32, st = C; the renderer's texel-major planes [B][C/32][h][w][32] have
 * sq = h*w*32, st = 32.  img (NULL: none) [B][C][n][n], c and out [B][C][2n][2n]; the same sums
 * as nfi_syn_up_add_forward.  The synthesis network's skip image runs channels-last and its last
 * image is written texel-major: the renderer reads it with no conversion pass.  C % 4 == 0, all
 * strides multiples of 4. */
int32_t nfi_syn_up_add_forward_strided(const float* img, const int64_t* img_strides, const float* c,
                                       const int64_t* c_strides, const float* bias, float* out,
                                       const int64_t* out_strides, int32_t B, int32_t C, int32_t n, void* stream);

/* Adjoint of upsample2d with the same strided layouts: g [B][C][2n][2n] -> gimg [B][C][n][n]. */
int32_t nfi_syn_up_backward_strided(const float* g, const int64_t* g_strides, float* gimg, const int64_t* gimg_strides,
                                    int32_t B, int32_t C, int32_t n, void* stream);

/* Backward of x * s[p] (stylegan.py:130 modulation): gx = g * s[p] (gx may be NULL),
 * ds[p] = sum_hw g * x (overwritten).  HW % 4 == 0. */
int32_t nfi_syn_scale_backward(const float* g, const float* x, const float* s, float* gx,
                               float* ds, int32_t P, int32_t HW, void* stream);

/* LPIPS distance head for one feature layer (lpips 0.1 `LPIPS.forward` as wrapped by
 * lib/metrics.py:130-146): per pixel n(f) = f / (||f||_C + 1e-10), d = sum_c w[c] (n(f0)-n(f1))_c^2;
 * out[i] = mean_hw d (out [N] overwritten).  f0, f1 [N,C,HW]; inv0/inv1 [N*HW] receive
 * 1/(||f||+1e-10) for the backward. */
int32_t nfi_lpips_head_forward(const float* f0, const float* f1, const float* w, float* out,
                               float* inv0, float* inv1, int32_t N, int32_t C, int32_t HW,
                               void* stream);

/* d out / d f0 scaled by g[N]: gf0 [N,C,HW] (overwritten).  At a pixel whose f0 vector is all
 * zero the gradient is 0 (torch's autograd of normalize_tensor gives NaN there). */
int32_t nfi_lpips_head_backward(const float* g, const float* f0, const float* f1, const float* w,
                                const float* inv0, const float* inv1, float* gf0, int32_t N,
                                int32_t C, int32_t HW, void* stream);

/* The LPIPS trunk's first layer (vgg16.features[0:2], metrics.py:107): x [N,3,H,W] -> y = relu(conv3x3(x,
 * w [Co,3,3,3], padding 1) + bias[co]) [N,Co,H,W], a direct convolution with the epilogue (27 products
 * per output: bound by writing y).  W % 4 == 0. */
int32_t nfi_vgg_first_forward(const float* x, const float* w, const float* bias, float* y, int32_t N, int32_t Co,
                              int32_t H, int32_t W, void* stream);
/* The same on the LPIPS ScalingLayer's output (nshift / nscale [3], both NULL: none): the convolution of
 * (x - nshift[c]) / nscale[c] (metrics.py via lpips 0.1, ATen's operation order; zero padding of the
 * normalised image), also leaving each image's max of y in its split-f16 slots ymax (split_slot; zero on
 * entry, may be NULL): the x scale of the next layer's nfi_dconv3x3 without a maxima pass. */
int32_t nfi_vgg_first_forward_max(const float* x, const float* nshift, const float* nscale, const float* w,
                                  const float* bias, float* y, uint32_t* ymax, int32_t N, int32_t Co, int32_t H, int32_t W,
                                  void* stream);
/* The backward through the ScalingLayer as well: gx = d(conv input) / nscale[c] (nscale NULL: none). */
int32_t nfi_vgg_first_backward_scaled(const float* gy, const float* y, const float* w, const float* nscale, float* gx,
                                      int32_t N, int32_t Co, int32_t H, int32_t W, void* stream);

/* Its backward to the image: gx [N,3,H,W] = conv_transpose(gy * (y > 0), w) (threshold_backward then
 * the data gradient; overwritten).  H % 16 == 0, W % 64 == 0. */
int32_t nfi_vgg_first_backward(const float* gy, const float* y, const float* w, float* gx, int32_t N, int32_t Co,
                               int32_t H, int32_t W, void* stream);

/* LPIPS VGG16 block epilogue (torchvision vgg16.features[:30] as lpips 0.1 runs it, metrics.py:107):
 * x [P, H, W] = a bias-free 3x3 convolution's output (P = N*C planes) -> y = relu(x + bias[c]);
 * when `pooled` is not NULL also pooled [P, H/2, W/2] = MaxPool2d(2, 2)(y).  Replaces the bias
 * add, nn.ReLU and nn.MaxPool2d passes of the conv blocks.  W % 4 == 0 (H even when pooling). */
int32_t nfi_vgg_bias_relu_forward(const float* x, const float* bias, float* y, float* pooled,
                                  int32_t P, int32_t C, int32_t H, int32_t W, void* stream);

/* Its backward: gx = (y > 0) * (gy + route(gpooled)), route = max_pool2d's backward (gradient to
 * the first maximum of each 2x2 window, row-major).  gy or gpooled may be NULL (not both). */
int32_t nfi_vgg_relu_backward(const float* gy, const float* gpooled, const float* y, float* gx,
                              int32_t P, int32_t H, int32_t W, void* stream);
/* The pooled form, also leaving each image's max |gx| (C planes per image) in its split-f16 slots gmax
 * (split_slot; zero on entry): the data gradient's nfi_dconv3x3 without a maxima pass. */
int32_t nfi_vgg_relu_backward_max(const float* gy, const float* gpooled, const float* y, float* gx, uint32_t* gmax,
                                  int32_t P, int32_t C, int32_t H, int32_t W, void* stream);

/* Winograd F(4x4, 3x3) convolution (stride 1, padding 1), the 3x3 convolutions of the LPIPS VGG16
 * trunk (lpips 0.1 via metrics.py:107) and of the synthesis layers (stylegan.py:130-145), i.e.
 * F.conv2d(x, w, padding=1) in fp32.  The layer is three transforms here around 36 independent
 * [Co x Ci] x [Ci x P] fp32 matrix products that the caller runs as one batched GEMM
 * (P = N * H/4 * W/4 tiles; M[k] = U[k] V[k], k = 0..35).  csrc/nfi_conv.hip.
 *
 * w [Co,Ci,3,3] -> U [36,Co,Ci]; flip != 0: the data-gradient weights U [36,Ci,Co] of rot180(w)
 * (conv_transpose2d(g, w, padding=1) == conv2d(g, rot180(w) with channels swapped, padding=1)). */
int32_t nfi_wino_weight_transform(const float* w, float* U, int32_t Co, int32_t Ci, int32_t flip,
                                  void* stream);

/* x [N,C,H,W] (16-byte aligned, H and W multiples of 4) -> V [36,C,P]. */
int32_t nfi_wino_input_transform(const float* x, float* V, int32_t N, int32_t C, int32_t H, int32_t W,
                                 void* stream);

/* The same for x * scale[n][c] (scale [N,C]; NULL: 1): the style modulation of the synthesis
 * layers (stylegan.py:130) folded into the transform. */
int32_t nfi_wino_input_transform_scaled(const float* x, const float* scale, float* V, int32_t N, int32_t C,
                                        int32_t H, int32_t W, void* stream);

/* The transform of (y > 0) * g (threshold_backward of a ReLU output y, then the data-gradient
 * Winograd's input transform): g, y [N,C,H,W] -> V [36,C,P] without the masked gradient in memory. */
int32_t nfi_wino_input_transform_relu_grad(const float* g, const float* y, float* V, int32_t N, int32_t C, int32_t H,
                                           int32_t W, void* stream);

/* M [36,Co,P] -> y [N,Co,H,W].  bias == NULL: y = the convolution.  bias != NULL: y =
 * relu(conv + bias[co]) (the LPIPS VGG16 block epilogue, as nfi_vgg_bias_relu_forward) and, when
 * pooled != NULL, pooled [N,Co,H/2,W/2] = MaxPool2d(2, 2)(y). */
int32_t nfi_wino_output_transform(const float* M, const float* bias, float* y, float* pooled, int32_t N,
                                  int32_t Co, int32_t H, int32_t W, void* stream);

/* The data gradient of a modulated convolution conv(x * scale) finished in the output transform:
 * M [36,C,P] = the data-gradient products (d(x * scale) in the Winograd domain) -> gx [N,C,H,W] =
 * that * scale[n][c] (gx may be NULL) and ds [N,C] = sum_hw that * x (overwritten) — the
 * modulation backward (nfi_syn_scale_backward) without the intermediate. */
int32_t nfi_wino_output_transform_scaled_grad(const float* M, const float* x, const float* scale, float* gx,
                                              float* ds, int32_t N, int32_t C, int32_t H, int32_t W, void* stream);

/* The fused layer: input transform, the 36 products on the matrix cores (v_mfma_f32_16x16x4_f32,
 * accumulators resident for a 32-tile x 32-channel block) and the output transform in one kernel,
 * same epilogue contract as nfi_wino_output_transform.  Ua = nfi_wino_pack_weights(U) (the
 * per-lane MFMA operand layout [36][CoP/16][Ci/4][64], CoP = Co rounded up to 32, zero rows;
 * nfi_wino_packed_size floats).  Ci % 8 == 0, H and W multiples of 4, x and y 16-byte aligned. */
int64_t nfi_wino_packed_size(int32_t Co, int32_t Ci);
int32_t nfi_wino_pack_weights(const float* U, float* Ua, int32_t Co, int32_t Ci, void* stream);
/* nfi_wino_conv_fused_split: the same convolution (+ bias/ReLU/pool epilogue) with the products on the
 * f16 matrix cores (split-f16, fp32-level error): Uh, Ul, uinv = nfi_split16_pack of U [36][Co][Ci]
 * (batch 36).  A workgroup: 16 x 16 outputs of one image x 64 output channels, the K reduction in
 * chunks of 32 channels and the 36 products consumed by the output transform one Winograd row at a
 * time.  Ci % 32 == 0, Co % 64 == 0, H and W multiples of 16. */
int32_t nfi_wino_conv_fused_split(const float* x, const uint16_t* Uh, const uint16_t* Ul, const float* uinv,
                                  const float* bias, float* y, float* pooled, int32_t N, int32_t Ci, int32_t Co,
                                  int32_t H, int32_t W, void* stream);
int32_t nfi_wino_conv_fused(const float* x, const float* Ua, const float* bias, float* y, float* pooled,
                            int32_t N, int32_t Ci, int32_t Co, int32_t H, int32_t W, void* stream);

/* ---- Direct 3x3 convolution on the f16 matrix cores (csrc/nfi_dconv.hip), for the large-map layers
 * (F.conv2d(x, w, b, padding=1), lpips VGG16 via metrics.py:107, stylegan.py:130-145 shapes): the
 * products as the split-f16 GEMM's (fp32-level error), x's power-of-two scale PER IMAGE.
 * nfi_dconv_pack: w [Co][Ci][3][3] fp32 -> wp [2][9][Ci'/8][Co'][8] fp16 bits (hi planes, then lo) and
 *   w_inv [1]; flip = 0: the forward weight (Co' = Co, Ci' = Ci); flip = 1: the data gradient's
 *   w'[ci][co][ky][kx] = w[co][ci][2-ky][2-kx] (Co' = Ci, Ci' = Co).  Ci' % 8 == 0.  Once per frozen
 *   weight.
 * nfi_dconv3x3: y [N][Co][H][W] = conv3x3(x', w) with x' = x (relu_y NULL) or x where relu_y > 0
 *   (threshold_backward of the block's output: the data gradient through the ReLU), then, when bias
 *   is given, relu(y + bias) and, when pooled is given, pooled = MaxPool2d(2, 2)(y).  slots: each image's
 *   max |x| (nfi_absmax_slots of x, or the ymax of the dconv that produced x; read, not consumed).
 *   xscale (may be NULL; then no relu_y and no bias): [N][Ci], the convolution of x * xscale[n][c] (the
 *   synthesis layers' modulation, stylegan.py:130); slots then bound max |x xscale| per image
 *   (nfi_absmax_scaled_slots).
 *   ymax (may be NULL; zero on entry): each image's max |y| atomically maxed into its slots, the next
 *   layer's slots (a bound for pooled too).  Ci % 16 == 0, Co % 64 == 0, H % 8 == 0, W % 64 == 0; wp
 *   16-B aligned. */
int32_t nfi_dconv_pack(const float* w, int32_t Co, int32_t Ci, int32_t flip, uint16_t* wp, float* w_inv, void* stream);
int32_t nfi_absmax_scaled_slots(const float* x, const float* scale, int32_t N, int32_t C, int32_t HW, uint32_t* slots,
                                void* stream);
int32_t nfi_dconv3x3(const float* x, const float* xscale, const float* relu_y, const uint32_t* slots, const uint16_t* wp, const float* w_inv,
                     const float* bias, float* y, float* pooled, uint32_t* ymax, int32_t N, int32_t Ci, int32_t Co,
                     int32_t H, int32_t W, void* stream);

/* The 'vgg' inversion loss's augmented copies (run.py:720-767 augment_impl as optimize_iter calls
 * it, run.py:2211-2235): img [B][H][W][3] (the rendered / target image, channels last), grid
 * [B*K][Ho][Wo][2] (affine_grid of each copy's rotation / scale / translation, copy j = b*K + k)
 * -> out [B*K][3][Ho][Wo] = grid_sample(img[b] - shift, grid[j], bilinear, zeros,
 * align_corners=False) + shift (shift 1 for white-background datasets, else 0).  Replaces the
 * expand-to-K-copies + F.grid_sample of the reference. */
int32_t nfi_aug_sample_forward(const float* img, const float* grid, float* out, int32_t B, int32_t K, int32_t H,
                               int32_t W, int32_t Ho, int32_t Wo, float shift, void* stream);

/* Its adjoint summed over the K copies: gout [B*K][3][Ho][Wo] -> gimg [B][H][W][3] (overwritten),
 * gathered per input pixel (no atomics; grid_sampler_2d_backward's weights).  Each copy's grid
 * must be an affine function of the output pixel (F.affine_grid, as augment_impl builds it): the
 * output pixels that sample an input pixel are enumerated in the preimage of its neighbourhood
 * under that map (read off the grid's corners), so a non-affine grid would lose contributions. */
int32_t nfi_aug_sample_backward(const float* gout, const float* grid, float* gimg, int32_t B, int32_t K, int32_t H,
                                int32_t W, int32_t Ho, int32_t Wo, void* stream);

/* The augmentation's sampling grid: F.affine_grid(theta, [N, C, H, W], align_corners=False)
 * (run.py:749 in augment_impl, :720-767) for theta [N][2][3]: grid [N][H][W][2] =
 * theta[n] . (x_i, y_j, 1) with x_i = linspace(-1, 1, W)_i (W - 1) / W (y_j likewise), the
 * products summed in ATen's order (x, y, then the translation).  One launch instead of ATen's
 * linspace / base-grid / bmm sequence. */
int32_t nfi_aug_affine_grid(const float* theta, int32_t N, int32_t H, int32_t W, float* grid, void* stream);

/* ---- Split-f16 batched GEMM (csrc/nfi_gemm.hip): C[b] = A[b] . B[b] in fp32 on the f16 matrix cores
 * (v_mfma_f32_16x16x32_f16), each fp32 operand a power-of-two-scaled hi + lo fp16 pair and each
 * product lo.hi + hi.lo + hi.hi on an fp32 accumulator (fp32-level error).  Replaces the
 * torch.bmm (hipBLASLt fp32) of the Winograd products of the 3x3 convolutions (stylegan.py:130-145,
 * lpips VGG16 via metrics.py:107).
 * nfi_split16_pack: A [batch][per] -> hi, lo [batch][per] (fp16 bits) and a_inv [batch] = 2^-e, with
 *   the largest |A[b]| 2^e in [2^14, 2^15) (one workgroup per batch entry; frozen operands: once).
 * Maxima slots (b_max / vmax / slots below): NFI_SPLIT16_SLOT_WORDS uint32 (= nfi_split16_slot_words()):
 *   image i's running maximum of |B| in words [64 (i mod 256), 64 (i mod 256) + 64) (float bits), a
 *   completion counter in word 16384.  B's power-of-two scale is PER IMAGE, so an image's operand
 *   precision (and result) does not depend on the other images of its batch (sharded = unsharded).
 * nfi_wino_input_transform_max: nfi_wino_input_transform_scaled (scale may be NULL) or, with relu_y,
 *   the ReLU-masked gradient transform, also leaving each image's running maximum of |V| in its
 *   slots.  vmax must hold zeros on entry: a zeroed buffer, or one a split GEMM has consumed.
 * nfi_absmax_slots: the same per-image maxima of any x [nimg][per_image] (every used slot and the counter
 *   rewritten: no prior zeroing needed).
 * nfi_gemm_split16: A halves [batch][M][K], B [batch][K][N] fp32, b_max from one of the above, C
 *   [batch][M][N] fp32 (written); K a multiple of 32; column n of every B[b] belongs to image
 *   n / cols_per_image (cols_per_image divides N; the Winograd products: tiles per image; N: one image).
 *   The launch's last workgroup returns the used slots and the counter to zero (no memset before the
 *   next producer).
 * nfi_gemm_split16_shared_a: the same with ONE A [M][K] (and a_inv[0]) for every batch entry, batch
 *   entry b being image b — the up-sampling convolutions' 9-tap weight matrix against each image
 *   (stylegan.py:99-101) — and K split in ksplit ranges when ksplit > 1 (few output tiles, long K: the
 *   data gradient W9^T dP), the partial products in work [ksplit][batch][M][N] summed in order
 *   (deterministic). */
#define NFI_SPLIT16_SLOT_WORDS 16385
int32_t nfi_split16_slot_words(void);
int32_t nfi_split16_pack(const float* A, int32_t batch, int64_t per, uint16_t* Ah, uint16_t* Al, float* a_inv,
                         void* stream);
int32_t nfi_wino_input_transform_max(const float* x, const float* scale, const float* relu_y, float* V,
                                     uint32_t* vmax, int32_t N, int32_t C, int32_t H, int32_t W, void* stream);
int32_t nfi_absmax_slots(const float* x, int32_t nimg, int64_t per_image, uint32_t* slots, void* stream);
int32_t nfi_gemm_split16(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                         const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                         int32_t cols_per_image, void* stream);
/* nfi_gemm_split16_ksplit: nfi_gemm_split16 with K split in ksplit ranges (few output tiles: the
 * 512-channel Winograd products at 8^2 / 16^2 maps), partials in work [ksplit][batch][M][N] summed in
 * order (deterministic). */
int32_t nfi_gemm_split16_ksplit(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                                const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                                int32_t cols_per_image, int32_t ksplit, float* work, void* stream);
int32_t nfi_gemm_split16_shared_a(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                                  const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                                  int32_t ksplit, float* work, void* stream);

/* AttentionMapper conditional norm + activation (generator.py:42-60 ConditionalLayerNorm, then the
 * leaky ReLU of :173-178): x = lrelu(beta + gamma1 * layer_norm(h), 0.2) per row of C channels
 * (C <= 1024; layer_norm without affine, eps 1e-5; gamma1 = 1 + gamma, beta with row stride ld,
 * h and x contiguous [B][C]); stats [B][2] = (mean, rstd) for the backward, which writes d h,
 * d gamma1 and d beta ([B][C] contiguous). */
int32_t nfi_syn_cond_norm_act_forward(const float* h, const float* gamma1, const float* beta, int32_t B, int32_t C,
                                      int32_t ld, float* x, float* stats, void* stream);
int32_t nfi_syn_cond_norm_act_backward(const float* gx, const float* h, const float* gamma1, const float* beta,
                                       const float* stats, int32_t B, int32_t C, int32_t ld, float* dh,
                                       float* dgamma1, float* dbeta, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NFI_PRODUCER_H */
