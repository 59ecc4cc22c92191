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
#include "nfi_host.h"
#include "../../include/nfi_producer.h"

namespace nfi {
namespace wino {

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

// grid (ceil(P / 256), C)
__global__ void __launch_bounds__(256) input_kernel(const float* __restrict__ x, float* __restrict__ V,
                                                    int C, int H, int W, int TW, int T, int64_t P) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (p >= P) return;
  const int n = (int)(p / T);
  const int t = (int)(p - (int64_t)n * T);
  const int ty = t / TW, tx = t - ty * TW;
  const float* xp = x + ((int64_t)n * C + c) * H * W;
  const int x0 = 4 * tx;
  float d[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int y = 4 * ty - 1 + r;
    if (y < 0 || y >= H) {
#pragma unroll
      for (int j = 0; j < 6; ++j) d[r][j] = 0.f;
      continue;
    }
    const float* row = xp + (int64_t)y * W;
    const float4 m = *reinterpret_cast<const float4*>(row + x0);
    d[r][0] = x0 > 0 ? row[x0 - 1] : 0.f;
    d[r][1] = m.x;
    d[r][2] = m.y;
    d[r][3] = m.z;
    d[r][4] = m.w;
    d[r][5] = x0 + 4 < W ? row[x0 + 4] : 0.f;
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
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float o[6];
    bt_col(s[r], o);
#pragma unroll
    for (int j = 0; j < 6; ++j) __builtin_nontemporal_store(o[j], out + (r * 6 + j) * plane);
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
    for (int j = 0; j < 6; ++j) m[r][j] = __builtin_nontemporal_load(src + (r * 6 + j) * plane);
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

int32_t nfi_wino_input_transform(const float* x, float* V, int32_t N, int32_t C, int32_t H, int32_t W,
                                 void* stream) {
  NFI_REQUIRE(x && V, "wino_input_transform: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && C <= 65535 && H >= 4 && W >= 4 && H % 4 == 0 && W % 4 == 0,
              "wino_input_transform: bad shape (H, W multiples of 4)");
  NFI_REQUIRE(((uintptr_t)x & 15) == 0, "wino_input_transform: x must be 16-byte aligned");
  const int TW = W / 4, T = (H / 4) * TW;
  const int64_t P = (int64_t)N * T;
  hipLaunchKernelGGL(input_kernel, dim3((unsigned)((P + 255) / 256), C), dim3(256), 0,
                     (hipStream_t)stream, x, V, C, H, W, TW, T, P);
  NFI_CHECK_LAUNCH("wino input_kernel");
  return NFI_OK;
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

}  // extern "C"
