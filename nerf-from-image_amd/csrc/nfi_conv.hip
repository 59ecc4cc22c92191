// Winograd F(4x4, 3x3) convolution transforms for gfx950 (stride 1, padding 1, NCHW fp32).
//
//   y = A^T [ (G g G^T) (.) (B^T d B) ] A      per 4x4 output tile, 6x6 input patch
//
// The 36 element-wise products of a layer form 36 independent [Co x Ci] x [Ci x P] matrix
// products (P = N * H/4 * W/4 tiles), which run as one batched fp32 GEMM on the matrix cores
// (hipBLASLt through PyTorch-ROCm: 100-137 TFLOP/s measured on these shapes).  This file holds
// the memory-bound parts around it:
//
//   weight_kernel   w [Co][Ci][3][3] -> U [36][Co][Ci]; or, for the data gradient (the
//                   transposed convolution = correlation with rot180(w), channels swapped),
//                   U [36][Ci][Co].  Once per frozen weight.
//   input_kernel    x [N][C][H][W] -> V [36][C][P]: one lane per (channel, tile); each patch row
//                   is a float4 plus its two neighbour columns (L1-served); 36 coalesced stores.
//   output_kernel   M [36][Co][P] -> y [N][Co][H][W] (+ bias, ReLU, 2x2 max pool fused: the
//                   LPIPS VGG16 block epilogue, nfi_vgg_bias_relu_forward's contract — a 4x4
//                   tile holds whole pool windows).
//
// Winograd minimal filtering (Lavin & Gray 2016).  Reference semantics replaced:
// F.conv2d(x, w, padding=1) as the LPIPS VGG16 trunk (lpips 0.1 via lib/metrics.py:107) and the
// synthesis layers (models/stylegan.py:130-145) call it; the reference runs fp32 with TF32 off
// (run.py:59-60), which this keeps (fp32 transforms, fp32 GEMM).
#include "nfi_common.h"
#include "nfi_host.h"
#include "../../include/nfi_producer.h"

namespace nfi {
namespace wino {

// V and M stream through HBM once each; NFI_WINO_NT 1 marks those accesses nontemporal
#ifndef NFI_WINO_NT
#define NFI_WINO_NT 1
#endif
__device__ __forceinline__ void st_stream(float v, float* p) {
#if NFI_WINO_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ float ld_stream(const float* p) {
#if NFI_WINO_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

// Interpolation points 0, 1, -1, 2, -1/2 and infinity: in fp32 this point set has about half
// the transform rounding error of the usual 0, +-1, +-2 (measured by emulation: 2.4e-6 vs 4.3e-6
// mean, 8e-6 vs 2.8e-5 max of a 256-channel tile relative to its largest output); the input
// transform's coefficients stay exact binary fractions.

// t = G g for a 3-vector g (G: 6x3)
__device__ __forceinline__ void g_col(const float g0, const float g1, const float g2, float* t) {
  t[0] = g0;
  t[1] = -(g0 + g1 + g2) * (1.f / 3.f);
  t[2] = (g0 - g1 + g2) * (1.f / 3.f);
  t[3] = (g0 + 2.f * g1 + 4.f * g2) * (1.f / 15.f);
  t[4] = (-16.f * g0 + 8.f * g1 - 4.f * g2) * (1.f / 15.f);
  t[5] = g2;
}

// t = B^T d for a 6-vector d
__device__ __forceinline__ void bt_col(const float* d, float* t) {
  t[0] = (d[0] - 2.f * d[2] + d[4]) + 1.5f * (d[1] - d[3]);
  t[1] = (d[4] - d[1]) - 2.5f * d[2] - 0.5f * d[3];
  t[2] = (d[1] + d[4]) + 0.5f * d[2] - 2.5f * d[3];
  t[3] = (d[4] - d[2]) + 0.5f * (d[3] - d[1]);
  t[4] = (d[4] - d[2]) + 2.f * (d[1] - d[3]);
  t[5] = (d[1] - 2.f * d[3] + d[5]) + 1.5f * (d[2] - d[4]);
}

// o = A^T m for a 6-vector m (A^T: 4x6)
__device__ __forceinline__ void at_col(const float* m, float* o) {
  const float a = m[1] + m[2], b = m[1] - m[2];
  o[0] = (m[0] + a) + (m[3] + m[4]);
  o[1] = b + 2.f * m[3] - 0.5f * m[4];
  o[2] = a + 4.f * m[3] + 0.25f * m[4];
  o[3] = (b + m[5]) + 8.f * m[3] - 0.125f * m[4];
}

// The 6x6 input patch of tile (ty, tx), zero outside the map (padding 1) or when !valid.
// Branch-free: every load is issued at a clamped, valid address and the padding is applied by
// selects afterwards, so the 18 loads stay in flight together (a per-row load-or-zero branch
// makes the compiler wait vmcnt(0) at each branch and serialises them).
__device__ __forceinline__ void load_patch(const float* __restrict__ xp, int H, int W, int ty, int tx,
                                           bool valid, float (&d)[6][6]) {
  const int x0 = 4 * tx;
  const int xl = max(x0 - 1, 0), xr = min(x0 + 4, W - 1);
  float4 m4[6];
  float lv[6], rv[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int yy = min(max(4 * ty - 1 + r, 0), H - 1);
    const float* row = xp + (int64_t)yy * W;
    m4[r] = *reinterpret_cast<const float4*>(row + x0);
    lv[r] = row[xl];
    rv[r] = row[xr];
  }
  const bool okl = valid && x0 > 0, okr = valid && x0 + 4 < W;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int yy = 4 * ty - 1 + r;
    const bool ok = valid && yy >= 0 && yy < H;
    d[r][0] = (ok && okl) ? lv[r] : 0.f;
    d[r][1] = ok ? m4[r].x : 0.f;
    d[r][2] = ok ? m4[r].y : 0.f;
    d[r][3] = ok ? m4[r].z : 0.f;
    d[r][4] = ok ? m4[r].w : 0.f;
    d[r][5] = (ok && okr) ? rv[r] : 0.f;
  }
}

__global__ void __launch_bounds__(256) weight_kernel(const float* __restrict__ w, float* __restrict__ U,
                                                     int Co, int Ci, int flip) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Co * Ci) return;
  const int co = i / Ci, ci = i - co * Ci;
  const float* g = w + (int64_t)i * 9;
  float k[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) k[j] = flip ? g[8 - j] : g[j];
  // rows of G g (per kernel column), then (G g) G^T
  float t[3][6];
#pragma unroll
  for (int b = 0; b < 3; ++b) g_col(k[b], k[3 + b], k[6 + b], t[b]);
  const int64_t plane = (int64_t)Co * Ci;
  const int64_t off = flip ? (int64_t)ci * Co + co : (int64_t)co * Ci + ci;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float u[6];
    g_col(t[0][a], t[1][a], t[2][a], u);
#pragma unroll
    for (int b = 0; b < 6; ++b) U[(a * 6 + b) * plane + off] = u[b];
  }
}

// grid (ceil(P / 256), C).  scale (optional, [N][C]): the transform of x * scale[n][c] (the
// modulation of the synthesis layers, stylegan.py:130, applied to the input of the convolution;
// the transform is linear, so the per-(image, channel) factor multiplies the 36 outputs)
// vmax (optional, 64 slots of float bits): the running maximum of |V| for the split-f16 product
// (nfi_gemm.hip), one atomic per workgroup into slot (x + y) % 64
__global__ void __launch_bounds__(256) input_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                                    const float* __restrict__ mask, float* __restrict__ V, int C,
                                                    int H, int W, int TW, int T, int64_t P,
                                                    unsigned* __restrict__ vmax) {
  const int64_t p0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  const bool live = p0 < P;
  if (!live && vmax == nullptr) return;
  const int64_t p = live ? p0 : P - 1;   // (lanes past P run a clamped tile and store nothing)
  const int n = (int)(p / T);
  const int t = (int)(p - (int64_t)n * T);
  const int ty = t / TW, tx = t - ty * TW;
  const float* xp = x + ((int64_t)n * C + c) * H * W;
  float d[6][6];
  load_patch(xp, H, W, ty, tx, true, d);
  if (mask != nullptr) {   // threshold_backward: x is a ReLU output's gradient, mask that output
    float mk[6][6];
    load_patch(mask + ((int64_t)n * C + c) * H * W, H, W, ty, tx, true, mk);
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int j = 0; j < 6; ++j) d[r][j] = mk[r][j] > 0.f ? d[r][j] : 0.f;
  }
  if (scale != nullptr) {
    const float sc = scale[(int64_t)n * C + c];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int j = 0; j < 6; ++j) d[r][j] *= sc;
  }
  // columns: s = B^T d (per column), then rows: v = s B
  float s[6][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], o[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = d[r][j];
    bt_col(col, o);
#pragma unroll
    for (int r = 0; r < 6; ++r) s[r][j] = o[r];
  }
  const int64_t plane = (int64_t)C * P;
  float* out = V + (int64_t)c * P + p;
  float m = 0.f;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float o[6];
    bt_col(s[r], o);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if (live) st_stream(o[j], out + (r * 6 + j) * plane);
      m = fmaxf(m, fabsf(o[j]));
    }
  }
  if (vmax != nullptr) {
    __shared__ float red[4];
    m = wave_max(live ? m : 0.f);
    if (lane_id() == 0) lds_st(red + (threadIdx.x >> 6), m);
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(vmax + (blockIdx.x + blockIdx.y) % 64,
                __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
  }
}

// grid (ceil(P / 256), Co).  mode 0: y = conv; mode 1: y = relu(conv + bias[co]) and, when
// pooled != nullptr, pooled = MaxPool2d(2, 2)(y).
__global__ void __launch_bounds__(256) output_kernel(const float* __restrict__ M, const float* __restrict__ bias,
                                                     float* __restrict__ y, float* __restrict__ pooled,
                                                     int Co, int H, int W, int TW, int T, int64_t P,
                                                     int mode) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int co = blockIdx.y;
  if (p >= P) return;
  const int n = (int)(p / T);
  const int t = (int)(p - (int64_t)n * T);
  const int ty = t / TW, tx = t - ty * TW;
  const int64_t plane = (int64_t)Co * P;
  const float* src = M + (int64_t)co * P + p;
  float m[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int j = 0; j < 6; ++j) m[r][j] = ld_stream(src + (r * 6 + j) * plane);
  // columns: s = A^T m (4x6), then rows: o = s A (4x4)
  float s[4][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], o[4];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = m[r][j];
    at_col(col, o);
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r][j] = o[r];
  }
  float o[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) at_col(s[r], o[r]);
  if (mode == 1) {
    const float b = bias[co];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[r][j] = fmaxf(o[r][j] + b, 0.f);
  }
  float* dst = y + (((int64_t)n * Co + co) * H + 4 * ty) * W + 4 * tx;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    *reinterpret_cast<float4*>(dst + (int64_t)r * W) = make_float4(o[r][0], o[r][1], o[r][2], o[r][3]);
  if (pooled != nullptr) {
    const int W2 = W >> 1, H2 = H >> 1;
    float* pd = pooled + (((int64_t)n * Co + co) * H2 + 2 * ty) * W2 + 2 * tx;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      *reinterpret_cast<float2*>(pd + (int64_t)r * W2) =
          make_float2(fmaxf(fmaxf(o[2 * r][0], o[2 * r][1]), fmaxf(o[2 * r + 1][0], o[2 * r + 1][1])),
                      fmaxf(fmaxf(o[2 * r][2], o[2 * r][3]), fmaxf(o[2 * r + 1][2], o[2 * r + 1][3])));
  }
}

// The data gradient of a modulated convolution (conv(x * s)) finished in the output transform:
// g' = the transform of M (d(x * s)), gx = g' s[n][c] and ds[n][c] += sum g' x — the scale
// backward (nfi_syn_scale_backward) without g' in memory.  ds zeroed by the caller; a wave whose
// tiles are all in one image adds one atomic, else one per lane.
__global__ void __launch_bounds__(256) output_scaled_kernel(const float* __restrict__ M, const float* __restrict__ x,
                                                            const float* __restrict__ sc, float* __restrict__ gx,
                                                            float* __restrict__ ds, int C, int H, int W, int TW, int T,
                                                            int64_t P) {
  const int64_t p0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  const bool live = p0 < P;
  const int64_t p = live ? p0 : P - 1;
  const int n = (int)(p / T);
  const int t = (int)(p - (int64_t)n * T);
  const int ty = t / TW, tx = t - ty * TW;
  const int64_t plane = (int64_t)C * P;
  const float* src = M + (int64_t)c * P + p;
  float m[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int j = 0; j < 6; ++j) m[r][j] = ld_stream(src + (r * 6 + j) * plane);
  const int64_t off = (((int64_t)n * C + c) * H + 4 * ty) * W + 4 * tx;
  float4 xv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) xv[r] = *reinterpret_cast<const float4*>(x + off + (int64_t)r * W);
  float s[4][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], o[4];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = m[r][j];
    at_col(col, o);
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r][j] = o[r];
  }
  float o[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) at_col(s[r], o[r]);
  const float sv = sc[(int64_t)n * C + c];
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    acc += (o[r][0] * xv[r].x + o[r][1] * xv[r].y) + (o[r][2] * xv[r].z + o[r][3] * xv[r].w);
    if (live && gx)
      *reinterpret_cast<float4*>(gx + off + (int64_t)r * W) =
          make_float4(o[r][0] * sv, o[r][1] * sv, o[r][2] * sv, o[r][3] * sv);
  }
  acc = live ? acc : 0.f;
  const int n0 = __shfl(n, 0), n63 = __shfl(n, 63);
  if (n0 == n63) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d);
    if ((threadIdx.x & 63) == 0) atomicAdd(ds + (int64_t)n * C + c, acc);
  } else if (live) {
    atomicAdd(ds + (int64_t)n * C + c, acc);
  }
}

// ---------------------------------------------------------------------------------------
// Fused layer: input transform, the 36 products and the output transform in one kernel, so V
// and M never leave the chip (the unfused path writes and re-reads 2.25x the input and the
// output through HBM).  Output-stationary: a workgroup owns FP = 32 tiles x FC = 32 output
// channels for all 36 products; wave w accumulates products 9w .. 9w+8 (9 x 2 x 2
// v_mfma_f32_16x16x4_f32 tiles = 144 accumulator registers).  K loop over the input channels
// in chunks of FK = 8: every thread loads one (channel, tile) 6x6 patch, transforms it and
// writes its 36 values to an LDS V image (double buffered, the next chunk's patch is loaded
// during the current chunk's MFMAs); the A operands (U) are pre-packed per lane
// (nfi_wino_pack_weights: one coalesced 256-B load per MFMA operand).  Epilogue: the
// accumulators go through LDS one 16-channel half at a time (36 x 16 x 32 floats, the V
// buffers' space) and each thread transforms two (channel, tile) outputs with the same bias /
// ReLU / max-pool epilogue as output_kernel.
// ---------------------------------------------------------------------------------------
constexpr int FP = 32, FC = 64, FK = 8;
constexpr int HB = FC / 16;                   // 16-channel MFMA row blocks per workgroup
constexpr int VIMG = 36 * FK * FP;            // floats per V image
typedef float f4v __attribute__((ext_vector_type(4)));

// U [36][Co][Ci] -> Ua [36][CoP/16][Ci/4][64] (lane l: row l & 15, k l >> 4 of a 16x4 A operand;
// rows past Co are zero)
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ U, float* __restrict__ Ua,
                                                   int Co, int Ci, int CB, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int l = (int)(i & 63);
  const int64_t q = i >> 6;
  const int KC4 = Ci >> 2;
  const int kc = (int)(q % KC4);
  const int64_t q2 = q / KC4;
  const int cb = (int)(q2 % CB);
  const int xi = (int)(q2 / CB);
  const int co = 16 * cb + (l & 15), ci = 4 * kc + (l >> 4);
  Ua[i] = co < Co ? U[((int64_t)xi * Co + co) * Ci + ci] : 0.f;
}

// B^T d B of a patch, written to V image slot (xi, row, col): dst[xi * FK * FP]
__device__ __forceinline__ void stage_patch(float (&d)[6][6], float* __restrict__ dst) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], o[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = d[r][j];
    bt_col(col, o);
#pragma unroll
    for (int r = 0; r < 6; ++r) d[r][j] = o[r];
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float o[6];
    bt_col(d[r], o);
#pragma unroll
    for (int j = 0; j < 6; ++j) lds_st(dst + (r * 6 + j) * (FK * FP), o[j]);
  }
}

// A^T m A of one tile plus the epilogue, stored to y (and pooled)
__device__ __forceinline__ void emit_tile(float (&m)[6][6], float b, int mode, float* __restrict__ dst, int W,
                                          float* __restrict__ pd, int W2) {
  float s[4][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], o[4];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = m[r][j];
    at_col(col, o);
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r][j] = o[r];
  }
  float o[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) at_col(s[r], o[r]);
  if (mode == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[r][j] = fmaxf(o[r][j] + b, 0.f);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    *reinterpret_cast<float4*>(dst + (int64_t)r * W) = make_float4(o[r][0], o[r][1], o[r][2], o[r][3]);
  if (pd != nullptr) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
      *reinterpret_cast<float2*>(pd + (int64_t)r * W2) =
          make_float2(fmaxf(fmaxf(o[2 * r][0], o[2 * r][1]), fmaxf(o[2 * r + 1][0], o[2 * r + 1][1])),
                      fmaxf(fmaxf(o[2 * r][2], o[2 * r][3]), fmaxf(o[2 * r + 1][2], o[2 * r + 1][3])));
  }
}

#ifndef NFI_WINO_ADEPTH
#define NFI_WINO_ADEPTH 3   // 1: the previous one-product-ahead A loads
#endif

// grid (ceil(P / FP), CoP / FC), 256 threads, one workgroup per CU (occupancy 1: 288
// accumulator registers per lane, the next chunk's A operands and patch prefetched a whole
// chunk ahead).  Ci % FK == 0.
__global__ void __launch_bounds__(256, 1) fused_kernel(const float* __restrict__ x, const float* __restrict__ Ua,
                                                       const float* __restrict__ bias, float* __restrict__ y,
                                                       float* __restrict__ pooled, int Ci, int Co, int H, int W,
                                                       int TW, int T, int64_t P, int CB, int mode, int nPB,
                                                       int nCB) {
  __shared__ __attribute__((aligned(16))) float lds[2 * VIMG];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  // XCD-aware block order: workgroup b runs on XCD b % 8; XCD x takes the contiguous range
  // [x * G / 8, (x + 1) * G / 8) of the (channel block, tile block) grid in channel-block-major
  // order, so the A operands of a channel block (36 x 64 x Ci floats) stay in that XCD's L2
  const int G = gridDim.x;                         // nPB * nCB rounded up to a multiple of 8
  const int logical = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int cbk = logical / nPB;
  if (cbk >= nCB) return;                          // padding workgroups
  const int64_t p0 = (int64_t)(logical - cbk * nPB) * FP;
  const int cb0 = cbk * HB;
  const int KC4 = Ci >> 2, nk = Ci / FK;
  // staging role: channel cl of the chunk, tile pl of the block
  const int pl = t & 31, cl = t >> 5;
  const int64_t ps = p0 + pl;
  const bool pvalid = ps < P;
  int sn = 0, sty = 0, stx = 0;
  if (pvalid) {
    sn = (int)(ps / T);
    const int tt = (int)(ps - (int64_t)sn * T);
    sty = tt / TW;
    stx = tt - sty * TW;
  }
  const int64_t HW = (int64_t)H * W;
  const float* xs = x + ((int64_t)sn * Ci + cl) * HW;
  // V image [36][FK][FP]; odd channel rows rotated by 16 columns so that the two k rows a
  // half-wave reads (ds_read_b32 lane groups of 32) fall in different banks
  float* vdst = lds + cl * FP + ((pl + 16 * (cl & 1)) & 31);
  const int kk = l >> 4, cc = l & 15;

  f4v acc[9][HB][2];
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int h = 0; h < HB; ++h)
#pragma unroll
      for (int g = 0; g < 2; ++g) acc[a][h][g] = f4v{0.f, 0.f, 0.f, 0.f};

  // A operands, one product ahead: [h][s], one float per lane each
  const float* ua = Ua + (((int64_t)(9 * w) * CB + cb0) * KC4) * 64 + l;
  auto load_a = [&](int xl, int c, float (&A)[HB][2]) {
#pragma unroll
    for (int h = 0; h < HB; ++h)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) A[h][s2] = ua[(((int64_t)xl * CB + h) * KC4 + 2 * c + s2) * 64];
  };

  float d[6][6];
  // A operands AD products ahead (ring slot = product index % AD; 9 % AD == 0 keeps the slot of
  // product (c, xl) a compile-time xl % AD): an L2 round trip under load outlasts one product's
  // 16 MFMAs, and at occupancy 1 no other wave covers it
  constexpr int AD = NFI_WINO_ADEPTH;
  static_assert(9 % AD == 0, "A-operand prefetch depth divides the 9 products of a wave");
  float an[AD][HB][2];
  load_patch(xs, H, W, sty, stx, pvalid, d);
#pragma unroll
  for (int u = 0; u < AD; ++u) load_a(u, 0, an[u]);
  stage_patch(d, vdst);
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    const int cur = c & 1;
    if (c + 1 < nk) load_patch(xs + (int64_t)(c + 1) * FK * HW, H, W, sty, stx, pvalid, d);
    const float* V = lds + cur * VIMG;
    float bn[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int g = 0; g < 2; ++g)
        bn[s2][g] = V[((9 * w) * FK + 4 * s2 + kk) * FP + ((16 * g + cc + 16 * (kk & 1)) & 31)];
#pragma unroll
    for (int xl = 0; xl < 9; ++xl) {
      const int xi = 9 * w + xl;
      float a[HB][2], b[2][2];
#pragma unroll
      for (int h = 0; h < HB; ++h)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[h][s2] = an[xl % AD][h][s2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int g = 0; g < 2; ++g) b[s2][g] = bn[s2][g];
      if (xl + AD < 9) load_a(xl + AD, c, an[xl % AD]);
      else if (c + 1 < nk) load_a(xl + AD - 9, c + 1, an[xl % AD]);
      if (xl + 1 < 9) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int g = 0; g < 2; ++g)
            bn[s2][g] = V[((xi + 1) * FK + 4 * s2 + kk) * FP + ((16 * g + cc + 16 * (kk & 1)) & 31)];
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int h = 0; h < HB; ++h)
#pragma unroll
          for (int g = 0; g < 2; ++g)
            acc[xl][h][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h][s2], b[s2][g], acc[xl][h][g], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < nk) stage_patch(d, vdst + (cur ^ 1) * VIMG);
    __syncthreads();
  }

  // epilogue, one 16-channel block at a time: M image [36][16][FP]
  const int W2 = W >> 1, H2 = H >> 1;
#pragma unroll
  for (int h = 0; h < HB; ++h) {
#pragma unroll
    for (int xl = 0; xl < 9; ++xl)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          lds[((9 * w + xl) * 16 + 4 * kk + i) * FP + 16 * g + cc] = acc[xl][h][g][i];
    __syncthreads();
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int col = (t >> 5) + 8 * rep;
      const int co = cbk * FC + 16 * h + col;
      const int64_t p = p0 + (t & 31);
      if (co < Co && p < P) {
        float m[6][6];
#pragma unroll
        for (int xi = 0; xi < 36; ++xi) m[xi / 6][xi % 6] = lds[(xi * 16 + col) * FP + (t & 31)];
        const int n = (int)(p / T);
        const int tt = (int)(p - (int64_t)n * T);
        const int ty = tt / TW, tx = tt - ty * TW;
        float* dst = y + (((int64_t)n * Co + co) * H + 4 * ty) * W + 4 * tx;
        float* pd = pooled ? pooled + (((int64_t)n * Co + co) * H2 + 2 * ty) * W2 + 2 * tx : nullptr;
        emit_tile(m, mode == 1 ? bias[co] : 0.f, mode, dst, W, pd, W2);
      }
    }
    __syncthreads();
  }
}

}  // namespace wino
}  // namespace nfi

using namespace nfi::wino;

extern "C" {

int32_t nfi_wino_weight_transform(const float* w, float* U, int32_t Co, int32_t Ci, int32_t flip,
                                  void* stream) {
  NFI_REQUIRE(w && U, "wino_weight_transform: null pointer");
  NFI_REQUIRE(Co > 0 && Ci > 0 && (int64_t)Co * Ci < (1ll << 31), "wino_weight_transform: bad shape");
  const int n = Co * Ci;
  hipLaunchKernelGGL(weight_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w, U, Co,
                     Ci, flip ? 1 : 0);
  NFI_CHECK_LAUNCH("wino weight_kernel");
  return NFI_OK;
}

int32_t nfi_wino_input_transform_scaled(const float* x, const float* scale, float* V, int32_t N, int32_t C,
                                        int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(x && V, "wino_input_transform: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && C <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_input_transform: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0, "wino_input_transform: x must be 16-byte aligned");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(input_kernel, dim3((unsigned)((P + 255) / 256), C), dim3(256), 0,
                     (hipStream_t)stream, x, scale, nullptr, V, C, H, W, TW, T, P, nullptr);
  NFI_CHECK_LAUNCH("wino input_kernel");
  return NFI_OK;
}

int32_t nfi_wino_input_transform_relu_grad(const float* g, const float* y, float* V, int32_t N, int32_t C, int32_t H,
                                           int32_t W, void* stream) {
  NFI_REQUIRE(g && y && V, "wino_input_transform_relu_grad: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && C <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_input_transform_relu_grad: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(((uintptr_t)g & 15) == 0 && ((uintptr_t)y & 15) == 0, "wino_input_transform_relu_grad: misaligned");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(input_kernel, dim3((unsigned)((P + 255) / 256), C), dim3(256), 0,
                     (hipStream_t)stream, g, nullptr, y, V, C, H, W, TW, T, P, nullptr);
  NFI_CHECK_LAUNCH("wino input_kernel");
  return NFI_OK;
}

int32_t nfi_wino_input_transform_max(const float* x, const float* scale, const float* relu_y, float* V,
                                     uint32_t* vmax, int32_t N, int32_t C, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(x && V && vmax, "wino_input_transform_max: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && C <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_input_transform_max: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0 && (relu_y == nullptr || ((uintptr_t)relu_y & 15) == 0),
              "wino_input_transform_max: misaligned");
  NFI_REQUIRE(hipMemsetAsync(vmax, 0, 64 * 4, (hipStream_t)stream) == hipSuccess, "wino_input_transform_max: memset");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(input_kernel, dim3((unsigned)((P + 255) / 256), C), dim3(256), 0,
                     (hipStream_t)stream, x, scale, relu_y, V, C, H, W, TW, T, P, (unsigned*)vmax);
  NFI_CHECK_LAUNCH("wino input_kernel");
  return NFI_OK;
}

int32_t nfi_wino_input_transform(const float* x, float* V, int32_t N, int32_t C, int32_t H, int32_t W,
                                 void* stream) {
  return nfi_wino_input_transform_scaled(x, nullptr, V, N, C, H, W, stream);
}

int32_t nfi_wino_output_transform(const float* M, const float* bias, float* y, float* pooled, int32_t N,
                                  int32_t Co, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(M && y, "wino_output_transform: null pointer");
  NFI_REQUIRE(N > 0 && Co > 0 && Co <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_output_transform: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(pooled == nullptr || bias != nullptr, "wino_output_transform: pooling needs the bias/ReLU epilogue");
  NFI_REQUIRE(((uintptr_t)y & 15) == 0 && (pooled == nullptr || ((uintptr_t)pooled & 7) == 0),
              "wino_output_transform: misaligned output");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(output_kernel, dim3((unsigned)((P + 255) / 256), Co), dim3(256), 0,
                     (hipStream_t)stream, M, bias, y, pooled, Co, H, W, TW, T, P, bias ? 1 : 0);
  NFI_CHECK_LAUNCH("wino output_kernel");
  return NFI_OK;
}

int32_t nfi_wino_output_transform_scaled_grad(const float* M, const float* x, const float* scale, float* gx,
                                              float* ds, int32_t N, int32_t C, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(M && x && scale && ds, "wino_output_transform_scaled_grad: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && C <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_output_transform_scaled_grad: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)gx & 15) == 0, "wino_output_transform_scaled_grad: misaligned");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(ds, 0, sizeof(float) * N * C, st) != hipSuccess) {
    nfi::set_error("wino_output_transform_scaled_grad: memset failed");
    return NFI_ELAUNCH;
  }
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(output_scaled_kernel, dim3((unsigned)((P + 255) / 256), C), dim3(256), 0, st, M, x, scale, gx,
                     ds, C, H, W, TW, T, P);
  NFI_CHECK_LAUNCH("wino output_scaled_kernel");
  return NFI_OK;
}

int32_t nfi_wino_pack_weights(const float* U, float* Ua, int32_t Co, int32_t Ci, void* stream) {
  NFI_REQUIRE(U && Ua, "wino_pack_weights: null pointer");
  NFI_REQUIRE(Co > 0 && Ci > 0 && Ci % 4 == 0, "wino_pack_weights: bad shape (Ci % 4 == 0)");
  const int CB = (Co + FC - 1) / FC * HB;
  const int64_t n = (int64_t)36 * CB * (Ci / 4) * 64;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, U, Ua,
                     Co, Ci, CB, n);
  NFI_CHECK_LAUNCH("wino pack_kernel");
  return NFI_OK;
}

int64_t nfi_wino_packed_size(int32_t Co, int32_t Ci) {
  if (Co <= 0 || Ci <= 0 || Ci % 4) return -1;
  return (int64_t)36 * ((Co + FC - 1) / FC * FC) * Ci;
}

int32_t nfi_wino_conv_fused(const float* x, const float* Ua, const float* bias, float* y, float* pooled,
                            int32_t N, int32_t Ci, int32_t Co, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(x && Ua && y, "wino_conv_fused: null pointer");
  NFI_REQUIRE(N > 0 && Ci > 0 && Ci % FK == 0 && Co > 0 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_conv_fused: bad shape (Ci % 8, H % 4, W % 4 must be 0)");
  NFI_REQUIRE(pooled == nullptr || bias != nullptr, "wino_conv_fused: pooling needs the bias/ReLU epilogue");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && (pooled == nullptr || ((uintptr_t)pooled & 7) == 0),
              "wino_conv_fused: misaligned tensors");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  const int CoP = (Co + FC - 1) / FC * FC;
  NFI_REQUIRE((P + FP - 1) / FP < (1ll << 31) && CoP / FC <= 65535, "wino_conv_fused: too large");
  // 1-D grid of nPB * nCB workgroups rounded up to a multiple of 8 (fused_kernel maps them to XCDs)
  const int64_t nPB = (P + FP - 1) / FP, nCB = CoP / FC;
  const int64_t G = (nPB * nCB + 7) / 8 * 8;
  NFI_REQUIRE(G < (1ll << 31), "wino_conv_fused: too large");
  hipLaunchKernelGGL(fused_kernel, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, x, Ua, bias, y, pooled,
                     Ci, Co, H, W, TW, T, P, CoP / 16, bias ? 1 : 0, (int)nPB, (int)nCB);
  NFI_CHECK_LAUNCH("wino fused_kernel");
  return NFI_OK;
}

}  // extern "C"
