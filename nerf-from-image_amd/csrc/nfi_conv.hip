// Winograd F(4x4, 3x3) convolution transforms for gfx950 (stride 1, padding 1, NCHW fp32).
//
//   y = A^T [ (G g G^T) (.) (B^T d B) ] A      per 4x4 output tile, 6x6 input patch
//
// The 36 element-wise products of a layer form 36 independent [Co x Ci] x [Ci x P] matrix
// products (P = N * H/4 * W/4 tiles), which run as one batched fp32-accurate GEMM on the f16 matrix
// cores — nfi's split-f16 product (nfi_gemm.hip, nfi_gemm_split16[_ksplit]: 200-256 TFLOP/s
// fp32-equivalent on these shapes; torch.bmm / hipBLASLt fp32 only with NFI_SPLIT16=0) — or, for the
// 64-channel layers, inside the fused kernel below (fp32 MFMAs).  This file holds the transforms
// around the products and the fused kernels:
//
//   weight_kernel   w [Co][Ci][3][3] -> U [36][Co][Ci]; or, for the data gradient (the
//                   transposed convolution = correlation with rot180(w), channels swapped),
//                   U [36][Ci][Co].  Once per frozen weight.
//   input_kernel    x [N][C][H][W] -> V [36][C][P]: one lane per (channel, tile); each patch row
//                   is a float4 plus its two neighbour columns (L1-served); 36 coalesced stores;
//                   optionally each image's max |V| for the split product's per-image B scale.
//   output_kernel   M [36][Co][P] -> y [N][Co][H][W] (+ bias, ReLU, 2x2 max pool fused: the
//                   LPIPS VGG16 block epilogue, nfi_vgg_bias_relu_forward's contract — a 4x4
//                   tile holds whole pool windows).
//
// Winograd minimal filtering (Lavin & Gray 2016).  Reference semantics replaced:
// F.conv2d(x, w, padding=1) as the LPIPS VGG16 trunk (lpips 0.1 via lib/metrics.py:107) and the
// synthesis layers (models/stylegan.py:130-145) call it; the reference runs fp32 with TF32 off
// (run.py:59-60), which this keeps (fp32 transforms, fp32 GEMM).
#include <type_traits>

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
// vmax (optional, the split-f16 product's per-image slots, split_slot in nfi_host.h): each image's
// running maximum of |V| (nfi_gemm.hip).  A workgroup inside one image: one atomic; one that straddles
// images (small maps, T < 256): the per-image maxima reduced in LDS, one atomic per image of the block
// (per-lane global atomics measured +0.9 ms per inversion step on the LPIPS 8^2-32^2 layers).
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
    m = live ? m : 0.f;
    const int64_t pb = (int64_t)blockIdx.x * 256;
    const int nb0 = (int)(pb / T), nb1 = (int)(min(pb + 255, P - 1) / T);
    if (nb0 == nb1) {   // (block-uniform)
      __shared__ float red[4];
      m = wave_max(m);
      if (lane_id() == 0) lds_st(red + (threadIdx.x >> 6), m);
      __syncthreads();
      if (threadIdx.x == 0)
        atomicMax(vmax + split_slot(nb0, blockIdx.x + blockIdx.y),
                  __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
    } else {   // (block-uniform) the block straddles images: per-image maxima in LDS, then one
               // global atomic per image of the block
      __shared__ unsigned ired[257];   // images of 256 consecutive columns: at most 256 / T + 1
      const int ni = nb1 - nb0 + 1;
      for (int i = threadIdx.x; i < ni; i += 256) ired[i] = 0u;
      __syncthreads();
      if (m > 0.f) atomicMax(ired + (n - nb0), __float_as_uint(m));
      __syncthreads();
      for (int i = threadIdx.x; i < ni; i += 256)
        if (ired[i] != 0u) atomicMax(vmax + split_slot(nb0 + i, blockIdx.x + blockIdx.y), ired[i]);
    }
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
#ifndef NFI_WINO_FC
#define NFI_WINO_FC 64   // output channels per workgroup: 64 (one workgroup per CU) or 32 (two)
#endif
constexpr int FP = 32, FC = NFI_WINO_FC, FK = 8;
static_assert(FC == 32 || FC == 64, "fused_kernel: 32 or 64 output channels per workgroup");
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

// stage_patch in pieces: B^T applied to columns [J0, J1), then rows [R0, R1) transformed and stored
// (NFI_WINO_INTERLEAVE: the next chunk's staging spread over the current chunk's products)
template <int J0, int J1>
__device__ __forceinline__ void stage_cols(float (&d)[6][6]) {
#pragma unroll
  for (int j = J0; j < J1; ++j) {
    float col[6], o[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) col[r] = d[r][j];
    bt_col(col, o);
#pragma unroll
    for (int r = 0; r < 6; ++r) d[r][j] = o[r];
  }
}
template <int R0, int R1>
__device__ __forceinline__ void stage_rows(float (&d)[6][6], float* __restrict__ dst) {
#pragma unroll
  for (int r = R0; r < R1; ++r) {
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

#ifndef NFI_WINO_INTERLEAVE
#define NFI_WINO_INTERLEAVE 0   // 1: the next chunk's patch staging inside products 3..8 of this chunk
#endif
#ifndef NFI_WINO_ADEPTH
#define NFI_WINO_ADEPTH 3   // 1: the previous one-product-ahead A loads
#endif

// grid (ceil(P / FP), CoP / FC), 256 threads, one workgroup per CU (occupancy 1: 288
// accumulator registers per lane, the next chunk's A operands and patch prefetched a whole
// chunk ahead).  Ci % FK == 0.
__global__ void __launch_bounds__(256, 64 / FC) fused_kernel(const float* __restrict__ x, const float* __restrict__ Ua,
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
#if NFI_WINO_INTERLEAVE
      // the next chunk's staging beside this product's MFMAs (its patch loads, issued at the top of
      // the chunk, have had three products to arrive; the other V buffer is free since the barrier)
      if (c + 1 < nk) {
        float* nv = vdst + (cur ^ 1) * VIMG;
        if (xl == 3) stage_cols<0, 2>(d);
        if (xl == 4) stage_cols<2, 4>(d);
        if (xl == 5) stage_cols<4, 6>(d);
        if (xl == 6) stage_rows<0, 2>(d, nv);
        if (xl == 7) stage_rows<2, 4>(d, nv);
        if (xl == 8) stage_rows<4, 6>(d, nv);
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
#if !NFI_WINO_INTERLEAVE
    if (c + 1 < nk) stage_patch(d, vdst + (cur ^ 1) * VIMG);
#endif
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

// ---------------------------------------------------------------------------------------
// Fused convolution on the f16 matrix cores (round 4): input transform -> 36 products -> output
// transform in one kernel, the products as the split-f16 GEMM's (hi + lo halves of
// power-of-two-scaled fp32 operands, three f16 products each, fp32 accumulation: csrc/nfi_gemm.hip).
// A workgroup owns a 4 x 4 block of tiles (16 x 16 outputs of one image) and 64 output channels
// (wave w: channels 16w..16w+15, one 16 x 16 MFMA block of (channel, tile)).  The order is the
// transpose of fused_kernel's: the Winograd elements e = (e1, e2) are the OUTER loop and the channel
// chunks of 32 the outermost, so each product's accumulators are consumed by the output transform
// as soon as they are complete — y = sum over chunks and e of A^T-weights x M_e is linear — and no
// 36-product accumulator set is ever live (fused_kernel: 288 registers, one wave per SIMD; here
// 64 output accumulators per lane).  Per chunk: the 32-channel 18 x 18 input region is staged in LDS
// (rows of 28 floats: the 16 interior columns as aligned float4 at column 4, the halo at 3 and 20);
// per e1, each thread forms row e1 of B^T d (from the 4-5 patch rows that row reads) and its six
// B-transformed values for 2 channels of one tile, splits them (one power of two per chunk from the
// region's largest |x|: |V| <= 49 max|x|) and writes them as the B operands of the six products
// (e1, 0..5); the 6 x 3 MFMAs per wave follow, their results are unscaled, taken through A^T along
// e2 and added into the 4 x 4 outputs with A^T's e1 weights.
// MEASURED SLOWER than fused_kernel (64->64 @128^2, 64 images: 0.68 vs 0.48-0.51 ms; scripts/wino_layers.py)
// though half its error (1e-6 vs 2e-6 of the largest output): the compiler keeps ~300 registers live
// (one wave per SIMD) and each Winograd row's A-operand loads and two barriers are exposed.  Kept
// behind NFI_FUSED_SPLIT=1 (conv.FUSED_SPLIT, default off) with its test.
#ifndef NFI_FSPLIT_OCC
#define NFI_FSPLIT_OCC 1   // workgroups per CU the register budget is set for (2: spills)
#endif
constexpr int XT = 16;                  // tiles per workgroup (4 x 4)
constexpr int XKC = 32;                 // channels per chunk
constexpr int XRW = 28;                 // LDS region row (floats): 112-B rows spread a half-wave's b128 reads
constexpr int XRH = 18;
constexpr int XREG = XKC * XRH * XRW;   // floats
constexpr int XVK = XKC + 8;            // halves per V row
constexpr int XVG = 6 * XT * XVK;       // halves per V group image

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma_h16(u4v a, u4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}
__device__ __forceinline__ unsigned short hbits(float v) { return __builtin_bit_cast(unsigned short, (_Float16)v); }
__device__ __forceinline__ float hval(unsigned short b) { return (float)__builtin_bit_cast(_Float16, b); }

// B^T row e1 applied down the 6 patch rows: t = sum_i B^T[e1][i] d[i] (bt_col's coefficients)
template <int E1>
__device__ __forceinline__ float bt_row(const float (&d)[6]) {
  if constexpr (E1 == 0) return (d[0] - 2.f * d[2] + d[4]) + 1.5f * (d[1] - d[3]);
  if constexpr (E1 == 1) return (d[4] - d[1]) - 2.5f * d[2] - 0.5f * d[3];
  if constexpr (E1 == 2) return (d[1] + d[4]) + 0.5f * d[2] - 2.5f * d[3];
  if constexpr (E1 == 3) return (d[4] - d[2]) + 0.5f * (d[3] - d[1]);
  if constexpr (E1 == 4) return (d[4] - d[2]) + 2.f * (d[1] - d[3]);
  return (d[1] - 2.f * d[3] + d[5]) + 1.5f * (d[2] - d[4]);
}
// A^T[o][e] (at_col's coefficients)
__device__ __forceinline__ constexpr float at_w(int o, int e) {
  return o == 0 ? (e == 5 ? 0.f : 1.f)
       : o == 1 ? (e == 0 ? 0.f : e == 1 ? 1.f : e == 2 ? -1.f : e == 3 ? 2.f : e == 4 ? -0.5f : 0.f)
       : o == 2 ? (e == 0 ? 0.f : e == 1 ? 1.f : e == 2 ? 1.f : e == 3 ? 4.f : e == 4 ? 0.25f : 0.f)
                : (e == 0 ? 0.f : e == 1 ? 1.f : e == 2 ? -1.f : e == 3 ? 8.f : e == 4 ? -0.125f : 1.f);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, int bytes) {
  const uint64_t pb = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pb >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

struct SplitConvArgs {
  const float* x;               // [N][Ci][H][W]
  const unsigned short* Uh;     // [36][Co][Ci] f16 bits (nfi_split16_pack of U)
  const unsigned short* Ul;
  const float* uinv;            // [36]
  const float* bias;            // [Co] or null (no epilogue)
  float* y;                     // [N][Co][H][W]
  float* pooled;                // [N][Co][H/2][W/2] or null
  int Ci, Co, H, W, BX, BY;     // BX, BY: 16 x 16 blocks per row / column
};

template <int E1>
__device__ __forceinline__ void split_e1(const float* __restrict__ reg, unsigned short* __restrict__ vh,
                                        unsigned short* __restrict__ vl, int t, int q, float sx) {
  const int ty = t >> 2, tx = t & 3;
  unsigned hw[6], lw[6];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float* base = reg + (2 * q + c) * (XRH * XRW) + (4 * ty) * XRW + 4 * tx + 3;
    float d[6][6];   // the patch (rows B^T[e1] does not read are dead loads, removed)
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const float* rp = base + i * XRW;
      const f4v m = *reinterpret_cast<const f4v*>(rp + 1);
      d[i][0] = rp[0];
      d[i][1] = m[0];
      d[i][2] = m[1];
      d[i][3] = m[2];
      d[i][4] = m[3];
      d[i][5] = rp[5];
    }
    float tr[6];   // row e1 of B^T d (stage_patch's first pass, one row of it)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const float col[6] = {d[0][j], d[1][j], d[2][j], d[3][j], d[4][j], d[5][j]};
      tr[j] = bt_row<E1>(col);
    }
    float v[6];    // (B^T d B)[e1][0..5]
    bt_col(tr, v);
#pragma unroll
    for (int e2 = 0; e2 < 6; ++e2) {
      const float a = v[e2] * sx;
      const unsigned short h = hbits(a), lo = hbits(a - hval(h));
      if (c == 0) {
        hw[e2] = h;
        lw[e2] = lo;
      } else {
        hw[e2] |= (unsigned)h << 16;
        lw[e2] |= (unsigned)lo << 16;
      }
    }
  }
#pragma unroll
  for (int e2 = 0; e2 < 6; ++e2) {
    // (lds_st keeps the compiler from pairing these into ds_write2 stores, which need the gap)
    lds_st(reinterpret_cast<unsigned*>(vh + (e2 * XT + t) * XVK + 2 * q), hw[e2]);
    lds_st(reinterpret_cast<unsigned*>(vl + (e2 * XT + t) * XVK + 2 * q), lw[e2]);
  }
}

template <int E1>
__device__ __forceinline__ void products_e1(const SplitConvArgs& g, const unsigned short* __restrict__ vh,
                                            const unsigned short* __restrict__ vl, const u4v (&ah)[6],
                                            const u4v (&al)[6], float fsc, float (&Y)[4][4][4]) {
  const int l = lane_id(), i16 = l & 15, kg = l >> 4;
  // lane (i16, kg): channel 4kg + r of the wave's 16, tile i16.  S = A^T along e2, folded in per
  // product (A^T is linear in its six inputs), then the e1 weights into the 4 x 4 outputs
  float S[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 0; o < 4; ++o) S[r][o] = 0.f;
#pragma unroll
  for (int e2 = 0; e2 < 6; ++e2) {
    const int rr = (e2 * XT + i16) * XVK + 8 * kg;
    const u4v bh = *reinterpret_cast<const u4v*>(vh + rr);
    const u4v bl = *reinterpret_cast<const u4v*>(vl + rr);
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma_h16(al[e2], bh, acc);   // small terms first
    acc = mfma_h16(ah[e2], bl, acc);
    acc = mfma_h16(ah[e2], bh, acc);
    const float f = g.uinv[6 * E1 + e2] * fsc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float m = acc[r] * f;
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const float w = at_w(o, e2);
        if (w != 0.f) S[r][o] = fmaf(w, m, S[r][o]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int oy = 0; oy < 4; ++oy) {
      const float w = at_w(oy, E1);
      if (w != 0.f) {
#pragma unroll
        for (int ox = 0; ox < 4; ++ox) Y[r][oy][ox] = fmaf(w, S[r][ox], Y[r][oy][ox]);
      }
    }
}

__global__ void __launch_bounds__(256, NFI_FSPLIT_OCC) fused_split_kernel(SplitConvArgs g) {
  __shared__ __attribute__((aligned(16))) float lds[XREG + XVG + 8];   // region, V hi + lo, 4 maxima
  float* reg = lds;
  unsigned short* vh = reinterpret_cast<unsigned short*>(lds + XREG);
  unsigned short* vl = vh + XVG;
  float* red = lds + XREG + XVG;
  const int tid = threadIdx.x, l = lane_id(), w = tid >> 6;
  const int blk = blockIdx.x;                      // (image, block row, block column)
  const int bx = blk % g.BX, by = (blk / g.BX) % g.BY, n = blk / (g.BX * g.BY);
  const int co0 = blockIdx.y * 64;
  const int H = g.H, W = g.W, Ci = g.Ci;
  const int64_t HW = (int64_t)H * W;
  const float* xn = g.x + (int64_t)n * Ci * HW;
  const int i16 = l & 15, kg = l >> 4;
  const int t = tid & 15, q = tid >> 4;            // V role: tile t, channels 2q, 2q+1 of the chunk
  float Y[4][4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) Y[r][a][b] = 0.f;
  // A operands: U[e][co0 + 16w + i16][chunk + 8kg .. +7] (byte offsets: lane uoff, product ue2)
  const int uoff = ((co0 + 16 * w + i16) * Ci + 8 * kg) * 2;
  const int ue2 = g.Co * Ci * 2;
  const __amdgpu_buffer_rsrc_t urs_h = wave_rsrc(g.Uh, 36 * ue2), urs_l = wave_rsrc(g.Ul, 36 * ue2);
  const __amdgpu_buffer_rsrc_t xrs = wave_rsrc(xn, (int)(Ci * HW * 4));
  for (int c0 = 0; c0 < Ci; c0 += XKC) {
    // ---- stage the 32-channel region: 576 rows of 4 float4 (9 per thread) + 2 halo floats ----
    // (all loads issued at clamped addresses before any is used; padding by selects afterwards)
    f4v rv[9];
    float hv[5];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int k = tid + 256 * i, r = k >> 2, ci = r / XRH, rr = r - ci * XRH;
      const int yy = min(max(16 * by - 1 + rr, 0), H - 1);
      rv[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                          xrs, ((c0 + ci) * (int)HW + yy * W + 16 * bx + 4 * (k & 3)) * 4, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = min(tid + 256 * i, 2 * XKC * XRH - 1), r = k >> 1, ci = r / XRH, rr = r - ci * XRH;
      const int yy = min(max(16 * by - 1 + rr, 0), H - 1);
      const int xx = (k & 1) ? min(16 * bx + 16, W - 1) : max(16 * bx - 1, 0);
      hv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, ((c0 + ci) * (int)HW + yy * W + xx) * 4, 0, 0));
    }
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int k = tid + 256 * i, r = k >> 2, ci = r / XRH, rr = r - ci * XRH;
      const int yy = 16 * by - 1 + rr;
      const f4v z = (yy >= 0 && yy < H) ? rv[i] : f4v{0.f, 0.f, 0.f, 0.f};
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(z[0]), fabsf(z[1])), fmaxf(fabsf(z[2]), fabsf(z[3]))));
      lds_st_fenced(reinterpret_cast<f4v*>(reg + (ci * XRH + rr) * XRW + 4 + 4 * (k & 3)), z);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = tid + 256 * i, r = min(k, 2 * XKC * XRH - 1) >> 1, ci = r / XRH, rr = r - ci * XRH;
      const int yy = 16 * by - 1 + rr;
      const int xx = (k & 1) ? 16 * bx + 16 : 16 * bx - 1;
      const float z = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? hv[i] : 0.f;
      mx = fmaxf(mx, fabsf(z));
      if (k < 2 * XKC * XRH) reg[(ci * XRH + rr) * XRW + ((k & 1) ? 20 : 3)] = z;
    }
    mx = wave_max(mx);
    if (l == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // one power of two for the chunk: 49 max|x| (the B^T row sums squared) to [2^14, 2^15)
    const float m49 = 49.f * mx;
    int ex = 15 - __builtin_amdgcn_frexp_expf(m49);
    ex = (m49 > 0.f && m49 < __builtin_inff()) ? min(max(ex, -120), 120) : 0;
    const float sx = __builtin_ldexpf(1.f, ex), isx = __builtin_ldexpf(1.f, -ex);
    auto group = [&](auto e1c) {
      constexpr int E1 = decltype(e1c)::value;
      split_e1<E1>(reg, vh, vl, t, q, sx);
      // the six products' A operands (L2-resident U halves), in flight across the barrier.  Buffer
      // loads (lane offset in a VGPR, product offset in an SGPR: global loads made the compiler hoist
      // all 36 products' 64-bit addresses out of the chunk loop), the offset through an empty
      // volatile asm that stays behind the previous barrier (no hoisting of later groups' loads)
      int sbase = 6 * E1 * ue2;
      asm volatile("" : "+s"(sbase));
      u4v ah[6], al[6];
#pragma unroll
      for (int e2 = 0; e2 < 6; ++e2) {
        const int so = sbase + e2 * ue2;
        ah[e2] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(urs_h, uoff + 2 * c0, so, 0));
        al[e2] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(urs_l, uoff + 2 * c0, so, 0));
      }
      __syncthreads();
      products_e1<E1>(g, vh, vl, ah, al, isx, Y);
      __syncthreads();
    };
    group(std::integral_constant<int, 0>{});
    group(std::integral_constant<int, 1>{});
    group(std::integral_constant<int, 2>{});
    group(std::integral_constant<int, 3>{});
    group(std::integral_constant<int, 4>{});
    group(std::integral_constant<int, 5>{});
  }
  // ---- epilogue: lane (i16, kg) holds channels co0 + 16w + 4kg + r of tile i16 ----
  const int ty = i16 >> 2, tx = i16 & 3;
  const int oy0 = 16 * by + 4 * ty, ox0 = 16 * bx + 4 * tx;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + 16 * w + 4 * kg + r;
    if (co >= g.Co) continue;
    float o[4][4];
    const float b = g.bias ? g.bias[co] : 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) o[a][c] = g.bias ? fmaxf(Y[r][a][c] + b, 0.f) : Y[r][a][c];
    float* dst = g.y + (((int64_t)n * g.Co + co) * H + oy0) * W + ox0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
      *reinterpret_cast<float4*>(dst + (int64_t)a * W) = make_float4(o[a][0], o[a][1], o[a][2], o[a][3]);
    if (g.pooled) {
      const int W2 = W >> 1, H2 = H >> 1;
      float* pd = g.pooled + (((int64_t)n * g.Co + co) * H2 + (oy0 >> 1)) * W2 + (ox0 >> 1);
#pragma unroll
      for (int a = 0; a < 2; ++a)
        *reinterpret_cast<float2*>(pd + (int64_t)a * W2) =
            make_float2(fmaxf(fmaxf(o[2 * a][0], o[2 * a][1]), fmaxf(o[2 * a + 1][0], o[2 * a + 1][1])),
                        fmaxf(fmaxf(o[2 * a][2], o[2 * a][3]), fmaxf(o[2 * a + 1][2], o[2 * a + 1][3])));
    }
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
  // (no memset: vmax holds zeros on entry — a zeroed buffer, or one a split GEMM has consumed, which
  //  returns its 64 slots and completion counter to zero; include/nfi_producer.h)
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

int32_t nfi_wino_conv_fused_split(const float* x, const uint16_t* Uh, const uint16_t* Ul, const float* uinv,
                                  const float* bias, float* y, float* pooled, int32_t N, int32_t Ci, int32_t Co,
                                  int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(x && Uh && Ul && uinv && y, "wino_conv_fused_split: null pointer");
  NFI_REQUIRE(N > 0 && Ci > 0 && Ci % XKC == 0 && Co > 0 && Co % 64 == 0 && H >= 16 && W >= 16 && H % 16 == 0 &&
                  W % 16 == 0,
              "wino_conv_fused_split: bad shape (Ci %% 32, Co %% 64, H %% 16, W %% 16 must be 0)");
  NFI_REQUIRE(pooled == nullptr || bias != nullptr, "wino_conv_fused_split: pooling needs the bias/ReLU epilogue");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && (pooled == nullptr || ((uintptr_t)pooled & 7) == 0) &&
                  ((uintptr_t)Uh & 15) == 0 && ((uintptr_t)Ul & 15) == 0,
              "wino_conv_fused_split: misaligned tensors");
  const int BX = W / 16, BY = H / 16;
  const int64_t nb = (int64_t)N * BX * BY;
  NFI_REQUIRE(nb < (1ll << 31) && Co / 64 <= 65535 && (int64_t)Ci * H * W * 4 < (1ll << 31) &&
                  (int64_t)36 * Co * Ci * 2 < (1ll << 31),
              "wino_conv_fused_split: too large (32-bit buffer offsets)");
  SplitConvArgs g{x, reinterpret_cast<const unsigned short*>(Uh), reinterpret_cast<const unsigned short*>(Ul), uinv,
                  bias, y, pooled, Ci, Co, H, W, BX, BY};
  hipLaunchKernelGGL(fused_split_kernel, dim3((unsigned)nb, (unsigned)(Co / 64)), dim3(256), 0, (hipStream_t)stream, g);
  NFI_CHECK_LAUNCH("wino fused_split_kernel");
  return NFI_OK;
}

}  // extern "C"
