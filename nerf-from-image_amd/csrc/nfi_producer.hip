// Memory-bound operators of the tri-plane producer (StyleGAN2 synthesis network,
// models/stylegan.py:293-490) fused for gfx950: everything between the convolutions.
// One pass over HBM per fused operator, float4 accesses on the contiguous NCHW planes, per-plane
// reductions folded into the same pass (wave shuffles + one atomic per 4096-element chunk).
// See include/nfi_producer.h for the contract and DESIGN.md ("Producer") for the traffic model.
#include "nfi_host.h"
#include "../../include/nfi_producer.h"

namespace nfi {
namespace syn {

constexpr int RED_CHUNK4 = 1024;   // float4 per reduction block (4 per thread, 256 threads)
constexpr float SLOPE = 0.2f;      // F.leaky_relu(x, 0.2) (stylegan.py:356)

__device__ __forceinline__ float act(float o, float d, float b, float gain) {
  // stylegan.py:145 (x * dcoefs), :350 (+ bias), :352 (mul_(act_gain)), :356 (leaky_relu)
  float z = __fmul_rn(__fadd_rn(__fmul_rn(o, d), b), gain);
  return z > 0.f ? z : __fmul_rn(z, SLOPE);
}

__device__ __forceinline__ float act_slope(float o, float d, float b) {
  return __fadd_rn(__fmul_rn(o, d), b) > 0.f ? 1.f : SLOPE;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float wave_absmax(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// block (256) sum -> *dst: stored when the plane is one block (gridDim.x == 1: no zero-fill
// launch before), else one atomic per block into the zero-filled *dst
__device__ __forceinline__ void block_sum_atomic(float v, float* dst) {
  __shared__ float part[4];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = (part[0] + part[1]) + (part[2] + part[3]);
    if (gridDim.x == 1) *dst = s;
    else atomicAdd(dst, s);
  }
}

__global__ void __launch_bounds__(256) act_fwd_kernel(const float4* __restrict__ o,
                                                      const float* __restrict__ d,
                                                      const float* __restrict__ bias,
                                                      float4* __restrict__ y, int64_t n4, int C,
                                                      int HW4, float gain) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int p = (int)(i / HW4);
  const float dp = d[p], b = bias[p % C];
  const float4 v = o[i];
  y[i] = make_float4(act(v.x, dp, b, gain), act(v.y, dp, b, gain), act(v.z, dp, b, gain),
                     act(v.w, dp, b, gain));
}

// grid (chunks, P): gz = g*gain*slope, go = gz*d, dd[p] += sum gz*o
__global__ void __launch_bounds__(256) act_bwd_kernel(const float4* __restrict__ g,
                                                      const float4* __restrict__ o,
                                                      const float* __restrict__ d,
                                                      const float* __restrict__ bias,
                                                      float4* go, float* __restrict__ dd, int C,
                                                      int HW4, float gain) {
  const int p = blockIdx.y;
  const float dp = d[p], b = bias[p % C];
  const int64_t base = (int64_t)p * HW4;
  float acc = 0.f;
  // branch-free loads (clamped index; a lane past the plane adds 0 and stores nothing)
  float4 gv[4], ov[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = min(blockIdx.x * RED_CHUNK4 + k * 256 + (int)threadIdx.x, HW4 - 1);
    gv[k] = g[base + j];
    ov[k] = o[base + j];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = blockIdx.x * RED_CHUNK4 + k * 256 + threadIdx.x;
    float4 gz;
    gz.x = gv[k].x * gain * act_slope(ov[k].x, dp, b);
    gz.y = gv[k].y * gain * act_slope(ov[k].y, dp, b);
    gz.z = gv[k].z * gain * act_slope(ov[k].z, dp, b);
    gz.w = gv[k].w * gain * act_slope(ov[k].w, dp, b);
    const float part = (gz.x * ov[k].x + gz.y * ov[k].y) + (gz.z * ov[k].z + gz.w * ov[k].w);
    acc += j < HW4 ? part : 0.f;
    if (j < HW4) go[base + j] = make_float4(gz.x * dp, gz.y * dp, gz.z * dp, gz.w * dp);
  }
  block_sum_atomic(acc, dd + p);
}

// grid (chunks, P): gx = g*s[p] (optional), ds[p] += sum g*x
__global__ void __launch_bounds__(256) scale_bwd_kernel(const float4* __restrict__ g,
                                                        const float4* __restrict__ x,
                                                        const float* __restrict__ s,
                                                        float4* __restrict__ gx,
                                                        float* __restrict__ ds, int HW4) {
  const int p = blockIdx.y;
  const float sp = s[p];
  const int64_t base = (int64_t)p * HW4;
  float acc = 0.f;
  // branch-free loads (clamped index; a lane past the plane adds 0 and stores nothing)
  float4 gv[4], xv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = min(blockIdx.x * RED_CHUNK4 + k * 256 + (int)threadIdx.x, HW4 - 1);
    gv[k] = g[base + j];
    xv[k] = x[base + j];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = blockIdx.x * RED_CHUNK4 + k * 256 + threadIdx.x;
    const float part = (gv[k].x * xv[k].x + gv[k].y * xv[k].y) + (gv[k].z * xv[k].z + gv[k].w * xv[k].w);
    acc += j < HW4 ? part : 0.f;
    if (gx && j < HW4) gx[base + j] = make_float4(gv[k].x * sp, gv[k].y * sp, gv[k].z * sp, gv[k].w * sp);
  }
  block_sum_atomic(acc, ds + p);
}

// [1,3,3,1] taps
__device__ __forceinline__ float k4(int i) { return (i == 0 || i == 3) ? 1.f : 3.f; }

// FIR (gain 4, pad 1) of the (2n+1)^2 transposed-conv output + epilogue; 4 outputs per thread
__global__ void __launch_bounds__(256) fir_up_act_kernel(const float* __restrict__ t,
                                                         const float* __restrict__ d,
                                                         const float* __restrict__ bias,
                                                         float4* __restrict__ o,
                                                         float4* __restrict__ y, int64_t n4,
                                                         int C, int n, float gain) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int W2 = 2 * n, T = 2 * n + 1, q4 = W2 >> 2;
  const int per = W2 * q4;
  const int p = (int)(i / per);
  const int rem = (int)(i - (int64_t)p * per);
  const int yy = rem / q4, x0 = (rem - yy * q4) * 4;
  const float* tp = t + (int64_t)p * T * T;
  // branch-free: all 28 loads at clamped addresses, out-of-range taps zeroed by selects (a
  // load-or-zero branch per tap makes the compiler wait for each load before the next)
  float v[4][7];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = min(max(yy - 1 + r, 0), T - 1);
#pragma unroll
    for (int j = 0; j < 7; ++j) v[r][j] = tp[row * T + min(max(x0 - 1 + j, 0), T - 1)];
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = yy - 1 + r;
    const bool rok = row >= 0 && row < T;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int col = x0 - 1 + j;
      v[r][j] = (rok && col >= 0 && col < T) ? v[r][j] : 0.f;
    }
    const float kr = k4(r);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc[k] += kr * ((v[r][k] + v[r][k + 3]) + 3.f * (v[r][k + 1] + v[r][k + 2]));
  }
  const float dp = d[p], b = bias[p % C];
  const float inv = 1.f / 16.f;
  const float4 ov = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
  o[i] = ov;
  y[i] = make_float4(act(ov.x, dp, b, gain), act(ov.y, dp, b, gain), act(ov.z, dp, b, gain),
                     act(ov.w, dp, b, gain));
}

// Stride-2 3x3 transposed convolution from its per-tap products: P [B][9][C][n][n] (tap k =
// 3 ky + kx of W9 x, one GEMM for all taps) -> t [B][C][2n+1][2n+1], t[Y][X] = sum over the taps
// with Y = 2 iy + ky, X = 2 ix + kx.  Row Y takes ky = Y&1 at iy = Y>>1 and, when Y is even, also
// ky = 2 at iy = Y/2 - 1 (the same for columns): at most 4 products per output, loaded at clamped
// addresses and masked (branch-free).
__global__ void __launch_bounds__(256) tap_scatter_kernel(const float* __restrict__ P,
                                                          float* __restrict__ t, int64_t total,
                                                          int C, int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int T = 2 * n + 1;
  const int64_t plane = i / (T * T);
  const int rem = (int)(i - plane * T * T);
  const int Y = rem / T, X = rem - Y * T;
  const int b = (int)(plane / C), c = (int)(plane - (int64_t)b * C);
  const int64_t nn = (int64_t)n * n, tap = (int64_t)C * nn;
  const float* Pc = P + ((int64_t)b * 9 * C + c) * nn;
  const int kya = Y & 1, iya = Y >> 1, kxa = X & 1, ixa = X >> 1;
  const bool ya = iya < n, yb = !(Y & 1) && iya >= 1, xa = ixa < n, xb = !(X & 1) && ixa >= 1;
  const int ra = min(iya, n - 1), rb = max(iya - 1, 0), ca = min(ixa, n - 1), cb = max(ixa - 1, 0);
  const float paa = Pc[(kya * 3 + kxa) * tap + ra * n + ca];
  const float pab = Pc[(kya * 3 + 2) * tap + ra * n + cb];
  const float pba = Pc[(6 + kxa) * tap + rb * n + ca];
  const float pbb = Pc[8 * tap + rb * n + cb];
  const float s = ((ya && xa ? paa : 0.f) + (ya && xb ? pab : 0.f)) + ((yb && xa ? pba : 0.f) + (yb && xb ? pbb : 0.f));
  t[i] = s;
}

// The same scatter fused with the FIR + epilogue (fir_up_act_kernel), for 2n >= 64: one workgroup
// per 16 x 64 output tile of one plane; the tile's products P (9 taps x 11 x 36) are staged in
// LDS with coalesced loads, the (16+3) x (64+3) transposed-conv values t are formed in LDS with
// tap_scatter_kernel's arithmetic and each thread filters 4 outputs with fir_up_act_kernel's (the
// two-kernel path's operations, up to FMA contraction), without t's round trip through HBM.
constexpr int UF_TY = 16, UF_TX = 64;
constexpr int UF_PY = UF_TY / 2 + 3, UF_PX = UF_TX / 2 + 4;   // 11 x 36 products per tap
constexpr int UF_RY = UF_TY + 3, UF_RX = UF_TX + 3;           // 19 x 67 t values
__global__ void __launch_bounds__(256) up_fir_act_kernel(const float* __restrict__ P, const float* __restrict__ d,
                                                         const float* __restrict__ bias, float4* __restrict__ o,
                                                         float4* __restrict__ y, int C, int n, float gain) {
  __shared__ float Ps[9][UF_PY][UF_PX];
  __shared__ float Ts[UF_RY][UF_RX + 1];
  const int W2 = 2 * n, T = 2 * n + 1;
  const int tiles_x = W2 / UF_TX;
  const int tile = blockIdx.x, p = blockIdx.y;              // p = b * C + c
  const int Y0 = (tile / tiles_x) * UF_TY, X0 = (tile % tiles_x) * UF_TX;
  const int b = p / C, c = p - b * C;
  const int64_t nn = (int64_t)n * n, tap = (int64_t)C * nn;
  const float* Pc = P + ((int64_t)b * 9 * C + c) * nn;
  const int iy0 = Y0 / 2 - 2, ix0 = X0 / 2 - 2;
  // all 14 loads of a thread in flight together (clamped element index, masked stores)
  constexpr int PN = 9 * UF_PY * UF_PX, PIT = (PN + 255) / 256;
  float pv[PIT];
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int k = min(it * 256 + (int)threadIdx.x, PN - 1);
    const int tp = k / (UF_PY * UF_PX), r = (k / UF_PX) % UF_PY, q = k % UF_PX;
    const int iy = iy0 + r, ix = ix0 + q;
    const bool in = iy >= 0 && iy < n && ix >= 0 && ix < n;
    const float v = Pc[tp * tap + (int64_t)min(max(iy, 0), n - 1) * n + min(max(ix, 0), n - 1)];
    pv[it] = in ? v : 0.f;
  }
#pragma unroll
  for (int it = 0; it < PIT; ++it) {
    const int k = it * 256 + threadIdx.x;
    if (k < PN) (&Ps[0][0][0])[k] = pv[it];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < UF_RY * UF_RX; k += 256) {
    const int r = k / UF_RX, q = k - r * UF_RX;
    const int Yt = Y0 - 1 + r, Xt = X0 - 1 + q;             // t coordinates (may be outside [0, 2n])
    float s = 0.f;
    if (Yt >= 0 && Yt < T && Xt >= 0 && Xt < T) {
      const int kya = Yt & 1, iya = Yt >> 1, kxa = Xt & 1, ixa = Xt >> 1;
      const bool ya = iya < n, yb = !(Yt & 1) && iya >= 1, xa = ixa < n, xb = !(Xt & 1) && ixa >= 1;
      const int ra = iya - iy0, rb = iya - 1 - iy0, ca = ixa - ix0, cb = ixa - 1 - ix0;
      const float paa = Ps[kya * 3 + kxa][ra][ca], pab = Ps[kya * 3 + 2][ra][cb];
      const float pba = Ps[6 + kxa][rb][ca], pbb = Ps[8][rb][cb];
      s = ((ya && xa ? paa : 0.f) + (ya && xb ? pab : 0.f)) + ((yb && xa ? pba : 0.f) + (yb && xb ? pbb : 0.f));
    }
    Ts[r][q] = s;
  }
  __syncthreads();
  const int r0 = threadIdx.x / (UF_TX / 4), x4 = (threadIdx.x % (UF_TX / 4)) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) v[j] = Ts[r0 + r][x4 + j];
    const float kr = k4(r);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += kr * ((v[k] + v[k + 3]) + 3.f * (v[k + 1] + v[k + 2]));
  }
  const float dp = d[p], bb = bias[c];
  const float inv = 1.f / 16.f;
  const float4 ov = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
  const int64_t i = ((int64_t)p * W2 * W2 + (int64_t)(Y0 + r0) * W2 + X0 + x4) / 4;
  o[i] = ov;
  y[i] = make_float4(act(ov.x, dp, bb, gain), act(ov.y, dp, bb, gain), act(ov.z, dp, bb, gain),
                     act(ov.w, dp, bb, gain));
}

// The backward of the up-sampling layer tail in one pass, for n % 32 == 0: the epilogue's backward
// (act_bwd_kernel: gz = g gain slope(o), go = gz d[p], dd[p] += sum gz o), the FIR adjoint
// (fir_up_bwd_kernel) and the tap gather (tap_gather_kernel) — one workgroup per 8 x 32 block of
// dP's (iy, ix) for all 9 taps of one plane: go (20 x 68, masked to 0 outside the plane) and gt
// (17 x 65) are formed in LDS with those kernels' arithmetic; go and gt never reach HBM.  dd is
// summed over each tile's own 16 x 64 block of the plane (one atomic per workgroup; zeroed by the
// caller).
constexpr int UB_TY = 8, UB_TX = 32;                                   // dP block (iy, ix)
constexpr int UB_GY = 2 * UB_TY + 4, UB_GX = 2 * UB_TX + 4;            // 20 x 68 go values
constexpr int UB_RY = 2 * UB_TY + 1, UB_RX = 2 * UB_TX + 1;            // 17 x 65 gt values
__global__ void __launch_bounds__(256) up_bwd_fused_kernel(const float* __restrict__ g, const float* __restrict__ o,
                                                           const float* __restrict__ d, const float* __restrict__ bias,
                                                           float* __restrict__ dP, float* __restrict__ dd, int C,
                                                           int n, float gain, unsigned* __restrict__ vmax) {
  __shared__ float Gs[UB_GY][UB_GX + 1];
  __shared__ float Rs[UB_RY][UB_RX + 1];
  __shared__ float part[4];
  __shared__ float pmax[4];
  const int W2 = 2 * n;
  const int tiles_x = n / UB_TX;
  const int tile = blockIdx.x, p = blockIdx.y;
  const int iy0 = (tile / tiles_x) * UB_TY, ix0 = (tile % tiles_x) * UB_TX;
  const int b = p / C, c = p - b * C;
  const float dp = d[p], bb = bias[c];
  const int64_t plane = (int64_t)p * W2 * W2;
  const int R0 = 2 * iy0 - 2, C0 = 2 * ix0 - 2;                        // go tile origin
  constexpr int GN = UB_GY * UB_GX, GIT = (GN + 255) / 256;
  float gv[GIT], ov[GIT];
#pragma unroll
  for (int it = 0; it < GIT; ++it) {
    const int k = min(it * 256 + (int)threadIdx.x, GN - 1);
    const int r = k / UB_GX, q = k - r * UB_GX;
    const int64_t a = plane + (int64_t)min(max(R0 + r, 0), W2 - 1) * W2 + min(max(C0 + q, 0), W2 - 1);
    gv[it] = g[a];
    ov[it] = o[a];
  }
  float acc = 0.f;
#pragma unroll
  for (int it = 0; it < GIT; ++it) {
    const int k = it * 256 + threadIdx.x;
    const int r = k / UB_GX, q = k - r * UB_GX;
    const int Y = R0 + r, X = C0 + q;
    const bool in = k < GN && Y >= 0 && Y < W2 && X >= 0 && X < W2;
    const float gz = gv[it] * gain * act_slope(ov[it], dp, bb);
    const bool own = in && r >= 2 && r < 2 + 2 * UB_TY && q >= 2 && q < 2 + 2 * UB_TX;
    acc += own ? gz * ov[it] : 0.f;
    if (k < GN) Gs[r][q] = in ? gz * dp : 0.f;
  }
  __syncthreads();
  // gt rows 2 iy0 .. 2 iy0 + 16, cols 2 ix0 .. 2 ix0 + 64 (fir_up_bwd_kernel's sums)
  for (int k = threadIdx.x; k < UB_RY * UB_RX; k += 256) {
    const int rr = k / UB_RX, cc = k - rr * UB_RX;
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float h = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) h += k4(q) * Gs[rr + 3 - a][cc + 3 - q];
      s += k4(a) * h;
    }
    Rs[rr][cc] = s * (1.f / 16.f);
  }
  // dd: block sum of the owned gz * o
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(dd + p, (part[0] + part[1]) + (part[2] + part[3]));
  // dP[tap][iy][ix] = gt[2 iy + ky][2 ix + kx]
  const int lx = threadIdx.x % UB_TX, ly = threadIdx.x / UB_TX;
  const int64_t nn = (int64_t)n * n;
  float* out = dP + ((int64_t)b * 9 * C + c) * nn + (int64_t)(iy0 + ly) * n + ix0 + lx;
  float mx = 0.f;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const float v = Rs[2 * ly + ky][2 * lx + kx];
      out[(ky * 3 + kx) * C * nn] = v;
      mx = fmaxf(mx, fabsf(v));
    }
  if (vmax != nullptr) {   // (block-uniform) the running maximum of |dP| for the split-f16 product
    mx = wave_absmax(mx);
    if ((threadIdx.x & 63) == 0) pmax[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(vmax + split_slot(b, blockIdx.x + blockIdx.y), __float_as_uint(fmaxf(fmaxf(pmax[0], pmax[1]), fmaxf(pmax[2], pmax[3]))));
  }
}

// Its adjoint's operand (the data gradient of the transposed convolution is W9^T dP): gt
// [B][C][2n+1][2n+1] -> dP [B][9][C][n][n], dP[3ky+kx][c][iy][ix] = gt[c][2iy+ky][2ix+kx] (always
// inside gt).  One thread per (b, c, iy, ix): its 3x3 window, 9 coalesced row stores.
__global__ void __launch_bounds__(256) tap_gather_kernel(const float* __restrict__ gt,
                                                         float* __restrict__ dP, int64_t total,
                                                         int C, int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t nn = (int64_t)n * n;
  const int64_t plane = i / nn;                  // b * C + c
  const int pix = (int)(i - plane * nn);
  const int iy = pix / n, ix = pix - iy * n;
  const int b = (int)(plane / C), c = (int)(plane - (int64_t)b * C);
  const int T = 2 * n + 1;
  const float* g = gt + plane * T * T + (2 * iy) * T + 2 * ix;
  float v[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) v[ky * 3 + kx] = g[ky * T + kx];
  float* d = dP + ((int64_t)b * 9 * C + c) * nn + pix;
#pragma unroll
  for (int k = 0; k < 9; ++k) d[k * C * nn] = v[k];
}

// adjoint FIR: gt[r][c] = sum_ij k_i k_j / 16 * go[r+1-i][c+1-j]
__global__ void __launch_bounds__(256) fir_up_bwd_kernel(const float* __restrict__ go,
                                                         float* __restrict__ gt, int64_t total,
                                                         int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int W2 = 2 * n, T = 2 * n + 1;
  const int p = (int)(i / (T * T));
  const int rem = (int)(i - (int64_t)p * T * T);
  const int r = rem / T, c = rem - r * T;
  const float* gp = go + (int64_t)p * W2 * W2;
  // branch-free (clamped loads, masked): see fir_up_act_kernel
  float g[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = min(max(r + 1 - a, 0), W2 - 1);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) g[a][bb] = gp[row * W2 + min(max(c + 1 - bb, 0), W2 - 1)];
  }
  float acc = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = r + 1 - a;
    float h = 0.f;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int col = c + 1 - bb;
      h += k4(bb) * ((col >= 0 && col < W2) ? g[a][bb] : 0.f);
    }
    acc += (row >= 0 && row < W2) ? k4(a) * h : 0.f;
  }
  gt[i] = acc * (1.f / 16.f);
}

// out[2n x 2n] = upsample2d(img[n x n]) + c + bias; 4 outputs per thread
__global__ void __launch_bounds__(256) up_add_kernel(const float* __restrict__ img,
                                                     const float4* __restrict__ cc,
                                                     const float* __restrict__ bias,
                                                     float4* __restrict__ out, int64_t n4, int C,
                                                     int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int W2 = 2 * n, q4 = W2 >> 2;
  const int per = W2 * q4;
  const int p = (int)(i / per);
  const int rem = (int)(i - (int64_t)p * per);
  const int yy = rem / q4, x0 = (rem - yy * q4) * 4;
  const float b = bias[p % C];
  float4 cv = cc[i];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (img) {
    const float* ip = img + (int64_t)p * n * n;
    const int q = yy >> 1;
    // rows: even yy=2q -> img[q-1]*1 + img[q]*3 ; odd yy=2q+1 -> img[q]*3 + img[q+1]*1
    const int r0 = (yy & 1) ? q : q - 1;
    const float w0 = (yy & 1) ? 3.f : 1.f, w1 = (yy & 1) ? 1.f : 3.f;
    const int m = x0 >> 1;
    // branch-free: clamped loads, out-of-range taps zeroed by selects (see fir_up_act_kernel)
    float v[2][4];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int row = min(max(r0 + rr, 0), n - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[rr][j] = ip[row * n + min(max(m - 1 + j, 0), n - 1)];
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int row = r0 + rr;
      const bool rok = row >= 0 && row < n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = m - 1 + j;
        v[rr][j] = (rok && col >= 0 && col < n) ? v[rr][j] : 0.f;
      }
      const float wr = rr == 0 ? w0 : w1;
      acc[0] += wr * (v[rr][0] + 3.f * v[rr][1]);
      acc[1] += wr * (3.f * v[rr][1] + v[rr][2]);
      acc[2] += wr * (v[rr][1] + 3.f * v[rr][2]);
      acc[3] += wr * (3.f * v[rr][2] + v[rr][3]);
    }
  }
  const float inv = 1.f / 16.f;
  out[i] = make_float4(acc[0] * inv + (cv.x + b), acc[1] * inv + (cv.y + b),
                       acc[2] * inv + (cv.z + b), acc[3] * inv + (cv.w + b));
}

// The same with channel-contiguous layouts (each tensor addressed by float4 strides: element
// (b, c, y, x) at b*sb + (c/32)*sq + (y*w + x)*st + c%32 floats, sq = 32 and st = C for
// channels-last [B][h][w][C], sq = h*w*32 and st = 32 for the renderer's texel-major planes
// [B][C/32][h][w][32]): the skip-image chain runs channels-last and its last image is written
// texel-major, the renderer's layout, with no conversion pass.  One thread per output pixel and
// 4 channels, up_add_kernel's arithmetic (C % 4 == 0).
struct Str4 {
  long long b, q, t;   // float4 units
};
__device__ __forceinline__ long long str4_at(const Str4& s, int b, int c4, long long pix) {
  return b * s.b + (c4 >> 3) * s.q + pix * s.t + (c4 & 7);
}
__global__ void __launch_bounds__(256) up_add_str_kernel(const float4* __restrict__ img, Str4 si,
                                                         const float4* __restrict__ cc, Str4 sc,
                                                         const float4* __restrict__ bias,
                                                         float4* __restrict__ out, Str4 so, int64_t total4, int C4,
                                                         int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int W2 = 2 * n;
  const int64_t pix = i / C4;
  const int c4 = (int)(i - pix * C4);
  const int64_t per = (int64_t)W2 * W2;
  const int b = (int)(pix / per);
  const int rem = (int)(pix - (int64_t)b * per);
  const int Y = rem / W2, X = rem - Y * W2;
  const float4 bv = bias[c4];
  const float4 cv = cc[str4_at(sc, b, c4, rem)];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (img) {
    const int q = Y >> 1;
    const int r0 = (Y & 1) ? q : q - 1;
    const float w0 = (Y & 1) ? 3.f : 1.f, w1 = (Y & 1) ? 1.f : 3.f;
    const int mm = X >> 1;
    const int ca = (X & 1) ? mm : mm - 1;                 // columns ca, ca + 1
    float4 v[2][2];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = r0 + rr, col = ca + j;
        const float4 t = img[str4_at(si, b, c4, (long long)min(max(row, 0), n - 1) * n + min(max(col, 0), n - 1))];
        const bool ok = row >= 0 && row < n && col >= 0 && col < n;
        v[rr][j] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const float wr = rr == 0 ? w0 : w1;
      // up_add_kernel: even X: (v[m-1] + 3 v[m]), odd X: (3 v[m] + v[m+1])
#define NFI_UPC(F) acc.F += wr * ((X & 1) ? (3.f * v[rr][0].F + v[rr][1].F) : (v[rr][0].F + 3.f * v[rr][1].F));
      NFI_UPC(x) NFI_UPC(y) NFI_UPC(z) NFI_UPC(w)
#undef NFI_UPC
    }
  }
  const float inv = 1.f / 16.f;
  out[str4_at(so, b, c4, rem)] = make_float4(acc.x * inv + (cv.x + bv.x), acc.y * inv + (cv.y + bv.y),
                                             acc.z * inv + (cv.z + bv.z), acc.w * inv + (cv.w + bv.w));
}

// up_bwd_kernel with the same strided layouts: g [B][C][2n][2n] -> gimg [B][C][n][n], 4 channels a thread
__global__ void __launch_bounds__(256) up_bwd_str_kernel(const float4* __restrict__ g, Str4 sg,
                                                         float4* __restrict__ gimg, Str4 sr, int64_t total4, int C4,
                                                         int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int W2 = 2 * n;
  const int64_t pix = i / C4;
  const int c4 = (int)(i - pix * C4);
  const int64_t nn = (int64_t)n * n;
  const int b = (int)(pix / nn);
  const int rem = (int)(pix - (int64_t)b * nn);
  const int q = rem / n, m = rem - q * n;
  float4 gv[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = min(max(2 * q - 1 + a, 0), W2 - 1);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
      gv[a][bb] = g[str4_at(sg, b, c4, (long long)row * W2 + min(max(2 * m - 1 + bb, 0), W2 - 1))];
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = 2 * q - 1 + a;
    float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int col = 2 * m - 1 + bb;
      const bool ok = col >= 0 && col < W2;
      h.x += k4(bb) * (ok ? gv[a][bb].x : 0.f);
      h.y += k4(bb) * (ok ? gv[a][bb].y : 0.f);
      h.z += k4(bb) * (ok ? gv[a][bb].z : 0.f);
      h.w += k4(bb) * (ok ? gv[a][bb].w : 0.f);
    }
    const bool rok = row >= 0 && row < W2;
    acc.x += rok ? k4(a) * h.x : 0.f;
    acc.y += rok ? k4(a) * h.y : 0.f;
    acc.z += rok ? k4(a) * h.z : 0.f;
    acc.w += rok ? k4(a) * h.w : 0.f;
  }
  const float inv = 1.f / 16.f;
  gimg[str4_at(sr, b, c4, rem)] = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
}

// gimg[q][m] = sum over rows {2q-1:1, 2q:3, 2q+1:3, 2q+2:1} x cols (same) / 16
__global__ void __launch_bounds__(256) up_bwd_kernel(const float* __restrict__ g,
                                                     float* __restrict__ gimg, int64_t total,
                                                     int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int W2 = 2 * n;
  const int p = (int)(i / (n * n));
  const int rem = (int)(i - (int64_t)p * n * n);
  const int q = rem / n, m = rem - q * n;
  const float* gp = g + (int64_t)p * W2 * W2;
  // branch-free (clamped loads, masked): see fir_up_act_kernel
  float gv[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = min(max(2 * q - 1 + a, 0), W2 - 1);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) gv[a][bb] = gp[row * W2 + min(max(2 * m - 1 + bb, 0), W2 - 1)];
  }
  float acc = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = 2 * q - 1 + a;
    float h = 0.f;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int col = 2 * m - 1 + bb;
      h += k4(bb) * ((col >= 0 && col < W2) ? gv[a][bb] : 0.f);
    }
    acc += (row >= 0 && row < W2) ? k4(a) * h : 0.f;
  }
  gimg[i] = acc * (1.f / 16.f);
}

// LPIPS head: one thread per pixel, channels strided by HW (coalesced across the wave)
constexpr float LP_EPS = 1e-10f;

__global__ void __launch_bounds__(256) lpips_fwd_kernel(const float* __restrict__ f0,
                                                        const float* __restrict__ f1,
                                                        const float* __restrict__ w,
                                                        float* __restrict__ out,
                                                        float* __restrict__ inv0,
                                                        float* __restrict__ inv1, int N, int C,
                                                        int HW) {
  const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = pix < (int64_t)N * HW;
  const int n = live ? (int)(pix / HW) : 0;
  const int hw = live ? (int)(pix - (int64_t)n * HW) : 0;
  float d = 0.f;
  if (live) {
    const float* a = f0 + (int64_t)n * C * HW + hw;
    const float* b = f1 + (int64_t)n * C * HW + hw;
    float ra = 0.f, rb = 0.f;
#pragma unroll 4
    for (int c = 0; c < C; ++c) {
      const float x = a[(int64_t)c * HW], y = b[(int64_t)c * HW];
      ra += x * x;
      rb += y * y;
    }
    const float ia = 1.f / (sqrtf(ra) + LP_EPS), ib = 1.f / (sqrtf(rb) + LP_EPS);
#pragma unroll 4
    for (int c = 0; c < C; ++c) {
      const float t = a[(int64_t)c * HW] * ia - b[(int64_t)c * HW] * ib;
      d += w[c] * t * t;
    }
    inv0[pix] = ia;
    inv1[pix] = ib;
    d *= 1.f / (float)HW;
  }
  if (HW % 64 == 0) {               // the whole wave is one image
    d = wave_sum(d);
    if ((threadIdx.x & 63) == 0 && live) atomicAdd(out + n, d);
  } else if (live) {
    atomicAdd(out + n, d);
  }
}

__global__ void __launch_bounds__(256) lpips_bwd_kernel(const float* __restrict__ g,
                                                        const float* __restrict__ f0,
                                                        const float* __restrict__ f1,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ inv0,
                                                        const float* __restrict__ inv1,
                                                        float* __restrict__ gf0, int N, int C,
                                                        int HW) {
  const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (int64_t)N * HW) return;
  const int n = (int)(pix / HW);
  const int hw = (int)(pix - (int64_t)n * HW);
  const int64_t off = (int64_t)n * C * HW + hw;
  const float* a = f0 + off;
  const float* b = f1 + off;
  const float ia = inv0[pix], ib = inv1[pix];
  const float s = 2.f * g[n] / (float)HW;
  // u_c = s w_c (a_c ia - b_c ib); grad_k = ia u_k - ia^2 (a_k / r) sum_c u_c a_c, r = ||a||
  float ua = 0.f, r2 = 0.f;
#pragma unroll 4
  for (int c = 0; c < C; ++c) {
    const float x = a[(int64_t)c * HW];
    const float u = s * w[c] * (x * ia - b[(int64_t)c * HW] * ib);
    ua += u * x;
    r2 += x * x;
  }
  const float r = sqrtf(r2);
  float* o = gf0 + off;
  if (r == 0.f) {   // all-zero feature vector: torch's sqrt backward gives 0*inf = NaN here; we give 0
    for (int c = 0; c < C; ++c) o[(int64_t)c * HW] = 0.f;
    return;
  }
  const float k2 = ia * ia * ua / r;
#pragma unroll 4
  for (int c = 0; c < C; ++c) {
    const float x = a[(int64_t)c * HW];
    const float u = s * w[c] * (x * ia - b[(int64_t)c * HW] * ib);
    o[(int64_t)c * HW] = ia * u - k2 * x;
  }
}

// One-read forms for C = WAVES * CPW channels: a workgroup of WAVES waves takes 64 pixels, wave j
// holds channels [j*CPW, (j+1)*CPW) of its lane's pixel in registers; the per-pixel channel sums
// (||f0||^2, ||f1||^2, then the weighted squared difference / the backward's two dot products)
// are wave partials combined through LDS in a fixed order.  f0 and f1 are read from HBM once
// (the loops above read them twice, and the second pass misses the caches at these sizes).
template <int LP_WAVES, int CPW>
__global__ void __launch_bounds__(64 * LP_WAVES) lpips_fwd_regs_kernel(const float* __restrict__ f0,
                                                              const float* __restrict__ f1,
                                                              const float* __restrict__ w,
                                                              float* __restrict__ out,
                                                              float* __restrict__ inv0,
                                                              float* __restrict__ inv1, int N, int HW) {
  constexpr int C = LP_WAVES * CPW;
  __shared__ float red[3][LP_WAVES][64];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t total = (int64_t)N * HW;
  const int64_t pix = (int64_t)blockIdx.x * 64 + l;
  const bool live = pix < total;
  const int64_t pc = live ? pix : total - 1;
  const int n = (int)(pc / HW), hw = (int)(pc - (int64_t)n * HW);
  const int64_t off = ((int64_t)n * C + wv * CPW) * HW + hw;
  float xa[CPW], xb[CPW];
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    xa[k] = f0[off + (int64_t)k * HW];
    xb[k] = f1[off + (int64_t)k * HW];
  }
  float ra = 0.f, rb = 0.f;
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    ra = fmaf(xa[k], xa[k], ra);
    rb = fmaf(xb[k], xb[k], rb);
  }
  red[0][wv][l] = ra;
  red[1][wv][l] = rb;
  __syncthreads();
  float RA = 0.f, RB = 0.f;
#pragma unroll
  for (int j = 0; j < LP_WAVES; ++j) {
    RA += red[0][j][l];
    RB += red[1][j][l];
  }
  const float ia = 1.f / (sqrtf(RA) + LP_EPS), ib = 1.f / (sqrtf(RB) + LP_EPS);
  float d = 0.f;
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    const float t = xa[k] * ia - xb[k] * ib;
    d += w[wv * CPW + k] * t * t;
  }
  red[2][wv][l] = d;
  __syncthreads();
  if (wv != 0) return;
  float D = 0.f;
#pragma unroll
  for (int j = 0; j < LP_WAVES; ++j) D += red[2][j][l];
  D *= 1.f / (float)HW;
  if (live) {
    inv0[pix] = ia;
    inv1[pix] = ib;
  }
  if (HW % 64 == 0) {               // the whole wave is one image
    D = wave_sum(D);
    if (l == 0 && live) atomicAdd(out + n, D);
  } else if (live) {
    atomicAdd(out + n, D);
  }
}

template <int LP_WAVES, int CPW>
__global__ void __launch_bounds__(64 * LP_WAVES) lpips_bwd_regs_kernel(const float* __restrict__ g,
                                                              const float* __restrict__ f0,
                                                              const float* __restrict__ f1,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ inv0,
                                                              const float* __restrict__ inv1,
                                                              float* __restrict__ gf0, int N, int HW) {
  constexpr int C = LP_WAVES * CPW;
  __shared__ float red[2][LP_WAVES][64];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t total = (int64_t)N * HW;
  const int64_t pix = (int64_t)blockIdx.x * 64 + l;
  const bool live = pix < total;
  const int64_t pc = live ? pix : total - 1;
  const int n = (int)(pc / HW), hw = (int)(pc - (int64_t)n * HW);
  const int64_t off = ((int64_t)n * C + wv * CPW) * HW + hw;
  float xa[CPW], xb[CPW];
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    xa[k] = f0[off + (int64_t)k * HW];
    xb[k] = f1[off + (int64_t)k * HW];
  }
  const float ia = inv0[pc], ib = inv1[pc];
  const float s = 2.f * g[n] / (float)HW;
  // u_c = s w_c (a_c ia - b_c ib); grad_k = ia u_k - ia^2 (a_k / r) sum_c u_c a_c, r = ||a||
  float ua = 0.f, r2 = 0.f;
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    xb[k] = s * w[wv * CPW + k] * (xa[k] * ia - xb[k] * ib);   // u_k (b is not needed again)
    ua += xb[k] * xa[k];
    r2 += xa[k] * xa[k];
  }
  red[0][wv][l] = ua;
  red[1][wv][l] = r2;
  __syncthreads();
  float UA = 0.f, R2 = 0.f;
#pragma unroll
  for (int j = 0; j < LP_WAVES; ++j) {
    UA += red[0][j][l];
    R2 += red[1][j][l];
  }
  if (!live) return;
  const float r = sqrtf(R2);
  // all-zero feature vector: torch's sqrt backward gives 0*inf = NaN here; we give 0
  const float k2 = r == 0.f ? 0.f : ia * ia * UA / r;
  const float sa = r == 0.f ? 0.f : ia;
  float* o = gf0 + off;
#pragma unroll
  for (int k = 0; k < CPW; ++k) o[(int64_t)k * HW] = sa * xb[k] - k2 * xa[k];
}

// ---------------------------------------------------------------------------------------
// The LPIPS trunk's first layer (vgg16.features[0:2]: 3 -> Co channels, 3x3, padding 1, + bias,
// ReLU) as a direct convolution with the epilogue: K = 27 products per output, so the layer is
// bound by writing its Co-channel output — one pass, instead of a library convolution (~17
// TFLOP/s on this shape) plus the epilogue pass.  One thread per 4 consecutive pixels of one row:
// the 3 x 3 x 6 input window (zero padding by selects), Co float4 stores.  The weights are
// wave-uniform (scalar loads).
// Backward: gx = conv_transpose(gy * (y > 0)) (threshold_backward then the data gradient), one
// workgroup per 16 x 64 pixel block: the masked gradient of FB channels at a time is staged in
// LDS with a 1-pixel halo, each thread accumulates its 4 pixels x 3 input channels.
// ---------------------------------------------------------------------------------------
// ymax (optional): each image's max of y (>= 0 after the ReLU) into its split-f16 slots (split_slot):
// the next layer's direct convolution (nfi_dconv3x3) takes its x scale from them, no maxima pass
__global__ void __launch_bounds__(256) vgg_first_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float4* __restrict__ y,
                                                            int64_t total, int Co, int H, int W,
                                                            unsigned* __restrict__ ymax, const float* __restrict__ nsh,
                                                            const float* __restrict__ nsc) {
  // nsh / nsc (optional, [3]): the LPIPS ScalingLayer (x - shift[c]) / scale[c] (lpips 0.1) applied to the
  // map's pixels as they load, in ATen's order (subtract, then a correctly rounded division); the zero
  // padding is the normalised image's, as the reference pads it
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = i0 < total;
  if (!live && ymax == nullptr) return;
  const int64_t i = live ? i0 : total - 1;   // (lanes past the end: a clamped pixel quad, no store)
  const int W4 = W / 4;
  const int64_t row = i / W4;                // n * H + yy
  const int x0 = (int)(i - row * W4) * 4;
  const int n = (int)(row / H), yy = (int)(row - (int64_t)n * H);
  float v[3][3][6];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* xc = x + ((int64_t)n * 3 + c) * H * W;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ry = yy - 1 + r;
      const float* xr = xc + (int64_t)min(max(ry, 0), H - 1) * W;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int cx = x0 - 1 + j;
        float t = xr[min(max(cx, 0), W - 1)];
        if (nsh != nullptr) t = __fdiv_rn(t - nsh[c], nsc[c]);
        v[c][r][j] = (ry >= 0 && ry < H && cx >= 0 && cx < W) ? t : 0.f;
      }
    }
  }
  float4* yo = y + (((int64_t)n * Co) * H + yy) * W4 + x0 / 4;
  const int64_t plane4 = (int64_t)H * W4;
  float ym = 0.f;
  for (int co = 0; co < Co; ++co) {
    const float* wc = w + co * 27;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float wv = wc[c * 9 + r * 3 + kx];
#pragma unroll
          for (int k = 0; k < 4; ++k) a[k] = fmaf(wv, v[c][r][k + kx], a[k]);
        }
    const float b = bias[co];
    const float4 o = make_float4(fmaxf(a[0] + b, 0.f), fmaxf(a[1] + b, 0.f), fmaxf(a[2] + b, 0.f), fmaxf(a[3] + b, 0.f));
    ym = fmaxf(ym, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
    if (live) yo[co * plane4] = o;
  }
  if (ymax != nullptr) {
    ym = live ? ym : 0.f;
    const int n0 = __builtin_amdgcn_readfirstlane(n), n63 = __builtin_amdgcn_readlane(n, 63);
    if (n0 == n63) {   // (wave-uniform) the wave inside one image: one atomic
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) ym = fmaxf(ym, __shfl_xor(ym, o));
      if ((threadIdx.x & 63) == 0) atomicMax(ymax + split_slot(n0, blockIdx.x * 4 + (threadIdx.x >> 6)), __float_as_uint(ym));
    } else if (live) {
      atomicMax(ymax + split_slot(n, threadIdx.x), __float_as_uint(ym));
    }
  }
}

constexpr int VF_TY = 16, VF_TX = 64, VF_FB = 4;   // pixel block, channels per LDS stage
// nsc (optional, [3]): the gradient leaves through the ScalingLayer's division (d x = g / scale[c], ATen's
// div backward)
__global__ void __launch_bounds__(256) vgg_first_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                            const float* __restrict__ w, float* __restrict__ gx,
                                                            int Co, int H, int W, const float* __restrict__ nsc) {
  __shared__ float M[VF_FB][VF_TY + 2][VF_TX + 3];
  const int tiles_x = W / VF_TX;
  const int Y0 = (blockIdx.x / tiles_x) * VF_TY, X0 = (blockIdx.x % tiles_x) * VF_TX;
  const int n = blockIdx.y;
  const int ty = threadIdx.x / (VF_TX / 4), tx4 = (threadIdx.x % (VF_TX / 4)) * 4;
  const int64_t HW = (int64_t)H * W;
  float acc[3][4] = {};
  constexpr int SN = VF_FB * (VF_TY + 2) * (VF_TX + 2), SIT = (SN + 255) / 256;
  for (int c0 = 0; c0 < Co; c0 += VF_FB) {
    // stage m = gy * (y > 0) of channels c0 .. c0+FB-1 over rows Y0-1 .. Y0+16, cols X0-1 .. X0+64
    float gv[SIT], yv[SIT];
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int k = min(it * 256 + (int)threadIdx.x, SN - 1);
      const int f = k / ((VF_TY + 2) * (VF_TX + 2)), rem = k - f * ((VF_TY + 2) * (VF_TX + 2));
      const int r = rem / (VF_TX + 2), q = rem - r * (VF_TX + 2);
      const int Y = min(max(Y0 - 1 + r, 0), H - 1), X = min(max(X0 - 1 + q, 0), W - 1);
      const int64_t a = ((int64_t)n * Co + min(c0 + f, Co - 1)) * HW + (int64_t)Y * W + X;
      gv[it] = gy[a];
      yv[it] = y[a];
    }
    __syncthreads();   // the previous stage's reads are done
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int k = it * 256 + threadIdx.x;
      if (k < SN) {
        const int f = k / ((VF_TY + 2) * (VF_TX + 2)), rem = k - f * ((VF_TY + 2) * (VF_TX + 2));
        const int r = rem / (VF_TX + 2), q = rem - r * (VF_TX + 2);
        const int Y = Y0 - 1 + r, X = X0 - 1 + q;
        const bool in = Y >= 0 && Y < H && X >= 0 && X < W && c0 + f < Co;
        M[f][r][q] = (in && yv[it] > 0.f) ? gv[it] : 0.f;
      }
    }
    __syncthreads();
    for (int f = 0; f < VF_FB && c0 + f < Co; ++f) {
      const float* wc = w + (c0 + f) * 27;
      // gx[ci][Y][X] += w[co][ci][ky][kx] * m[co][Y+1-ky][X+1-kx]
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        float mv[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) mv[j] = M[f][ty + 2 - ky][tx4 + j];   // X + 1 - kx - (X0 - 1) = tx4 + 2 - kx + k
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) {
            const float wv = wc[ci * 9 + ky * 3 + kx];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[ci][k] = fmaf(wv, mv[k + 2 - kx], acc[ci][k]);
          }
      }
    }
  }
#pragma unroll
  for (int ci = 0; ci < 3; ++ci) {
    if (nsc != nullptr) {
      const float sc = nsc[ci];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[ci][k] = __fdiv_rn(acc[ci][k], sc);
    }
    *reinterpret_cast<float4*>(gx + ((int64_t)n * 3 + ci) * HW + (int64_t)(Y0 + ty) * W + X0 + tx4) =
        make_float4(acc[ci][0], acc[ci][1], acc[ci][2], acc[ci][3]);
  }
}

// ---------------------------------------------------------------------------------------
// VGG16 block epilogue of the LPIPS trunk (torchvision vgg16.features as lpips 0.1 runs it):
// conv output x (MIOpen, no bias) -> y = ReLU(x + bias[c]) and, before a MaxPool2d(2, 2), the
// pooled map m = max over each 2x2 window of y, in one pass (torch: bias add, relu, max_pool2d =
// three passes).  One thread per 2x4 patch of y (two float4 rows, two pooled outputs).
// Backward: gx = (y > 0) * (gy + route(gm)), route = gm to the FIRST maximum of its window in
// row-major order (ATen max_pool2d's `val > maxval` scan), i.e. threshold_backward of the sum of
// the tap gradient and max_pool2d_backward — the three backward kernels in one.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) vgg_bias_relu_kernel(const float4* __restrict__ x,
                                                            const float* __restrict__ bias,
                                                            float4* __restrict__ y, int64_t n4, int C,
                                                            int HW4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float b = bias[(int)((i / HW4) % C)];
  const float4 v = x[i];
  y[i] = make_float4(fmaxf(v.x + b, 0.f), fmaxf(v.y + b, 0.f), fmaxf(v.z + b, 0.f), fmaxf(v.w + b, 0.f));
}

__device__ __forceinline__ int first_max4(float a, float b, float c, float d, float& m) {
  int k = 0;
  m = a;
  if (b > m) { m = b; k = 1; }
  if (c > m) { m = c; k = 2; }
  if (d > m) { m = d; k = 3; }
  return k;
}

// patches: P planes x (H/2) row pairs x (W/4) column quads
__global__ void __launch_bounds__(256) vgg_bias_relu_pool_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ y,
                                                                 float* __restrict__ m, int64_t npatch,
                                                                 int C, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npatch) return;
  const int W4 = W >> 2, H2 = H >> 1;
  const int qx = (int)(i % W4);
  const int64_t t = i / W4;
  const int ry = (int)(t % H2);
  const int64_t p = t / H2;
  const float b = bias[(int)(p % C)];
  const int64_t o0 = (p * H + 2 * ry) * W + 4 * qx;
  const float4 u = *reinterpret_cast<const float4*>(x + o0);
  const float4 v = *reinterpret_cast<const float4*>(x + o0 + W);
  const float4 yu = make_float4(fmaxf(u.x + b, 0.f), fmaxf(u.y + b, 0.f), fmaxf(u.z + b, 0.f), fmaxf(u.w + b, 0.f));
  const float4 yv = make_float4(fmaxf(v.x + b, 0.f), fmaxf(v.y + b, 0.f), fmaxf(v.z + b, 0.f), fmaxf(v.w + b, 0.f));
  *reinterpret_cast<float4*>(y + o0) = yu;
  *reinterpret_cast<float4*>(y + o0 + W) = yv;
  float m0, m1;
  first_max4(yu.x, yu.y, yv.x, yv.y, m0);
  first_max4(yu.z, yu.w, yv.z, yv.w, m1);
  *reinterpret_cast<float2*>(m + (p * H2 + ry) * (W >> 1) + 2 * qx) = make_float2(m0, m1);
}

__global__ void __launch_bounds__(256) vgg_relu_bwd_kernel(const float4* __restrict__ gy,
                                                           const float4* __restrict__ y,
                                                           float4* __restrict__ gx, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 g = gy[i], v = y[i];
  gx[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                      v.w > 0.f ? g.w : 0.f);
}

__global__ void __launch_bounds__(256) vgg_relu_pool_bwd_kernel(const float* __restrict__ gy,
                                                                const float* __restrict__ gm,
                                                                const float* __restrict__ y,
                                                                float* __restrict__ gx, int64_t npatch,
                                                                int H, int W, unsigned* __restrict__ gmax, int C) {
  // gmax (optional): each image's max |gx| (C planes per image) into its split-f16 slots, for the data
  // gradient's direct convolution (nfi_dconv3x3) without a maxima pass
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = i0 < npatch;
  if (!live && gmax == nullptr) return;
  const int64_t i = live ? i0 : npatch - 1;
  const int W4 = W >> 2, H2 = H >> 1;
  const int qx = (int)(i % W4);
  const int64_t t = i / W4;
  const int ry = (int)(t % H2);
  const int64_t p = t / H2;
  const int64_t o0 = (p * H + 2 * ry) * W + 4 * qx;
  const float4 yu = *reinterpret_cast<const float4*>(y + o0);
  const float4 yv = *reinterpret_cast<const float4*>(y + o0 + W);
  float4 gu = make_float4(0.f, 0.f, 0.f, 0.f), gv = gu;
  if (gy) {
    gu = *reinterpret_cast<const float4*>(gy + o0);
    gv = *reinterpret_cast<const float4*>(gy + o0 + W);
  }
  if (gm) {
    const float2 g2 = *reinterpret_cast<const float2*>(gm + (p * H2 + ry) * (W >> 1) + 2 * qx);
    float mm;
    const int k0 = first_max4(yu.x, yu.y, yv.x, yv.y, mm);
    const int k1 = first_max4(yu.z, yu.w, yv.z, yv.w, mm);
    // (g + 0 == g exactly: the unrouted entries keep the tap gradient unchanged)
    if (k0 == 0) gu.x += g2.x; else if (k0 == 1) gu.y += g2.x; else if (k0 == 2) gv.x += g2.x; else gv.y += g2.x;
    if (k1 == 0) gu.z += g2.y; else if (k1 == 1) gu.w += g2.y; else if (k1 == 2) gv.z += g2.y; else gv.w += g2.y;
  }
  const float4 ou = make_float4(yu.x > 0.f ? gu.x : 0.f, yu.y > 0.f ? gu.y : 0.f, yu.z > 0.f ? gu.z : 0.f,
                                yu.w > 0.f ? gu.w : 0.f);
  const float4 ov = make_float4(yv.x > 0.f ? gv.x : 0.f, yv.y > 0.f ? gv.y : 0.f, yv.z > 0.f ? gv.z : 0.f,
                                yv.w > 0.f ? gv.w : 0.f);
  if (live) {
    *reinterpret_cast<float4*>(gx + o0) = ou;
    *reinterpret_cast<float4*>(gx + o0 + W) = ov;
  }
  if (gmax != nullptr) {
    float m = fmaxf(fmaxf(fmaxf(fabsf(ou.x), fabsf(ou.y)), fmaxf(fabsf(ou.z), fabsf(ou.w))),
                    fmaxf(fmaxf(fabsf(ov.x), fabsf(ov.y)), fmaxf(fabsf(ov.z), fabsf(ov.w))));
    m = live ? m : 0.f;
    const int n = (int)(p / C);
    const int n0 = __builtin_amdgcn_readfirstlane(n), n63 = __builtin_amdgcn_readlane(n, 63);
    if (n0 == n63) {   // (wave-uniform) the wave inside one image: one atomic
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      if ((threadIdx.x & 63) == 0) atomicMax(gmax + split_slot(n0, blockIdx.x * 4 + (threadIdx.x >> 6)), __float_as_uint(m));
    } else if (live) {
      atomicMax(gmax + split_slot(n, threadIdx.x), __float_as_uint(m));
    }
  }
}

// ---------------------------------------------------------------------------------------
// The 'vgg' loss's augmented copies (run.py:720-767 augment_impl, as optimize_iter calls it at
// run.py:2211-2235): K copies of each image [B][H][W][3] resampled through their own affine grid
// [B*K][Ho][Wo][2] by grid_sample(bilinear, zeros, align_corners=False) after the white-background
// shift (img - shift, + shift after).  The arithmetic restates ATen's grid_sampler_2d (source index
// ((g + 1) * size - 1) / 2, floor corners, weights nw = (ix_se - ix)(iy_se - iy), ..., corners
// accumulated nw, ne, sw, se).  The image is read in place (no expanded contiguous copies).
// ---------------------------------------------------------------------------------------
struct Samp {
  float ix, iy;
  int x0, y0;
};
__device__ __forceinline__ Samp samp_at(const float* __restrict__ g, int W, int H) {
  Samp s;
  const float2 gv = *reinterpret_cast<const float2*>(g);
  s.ix = ((gv.x + 1.f) * (float)W - 1.f) / 2.f;
  s.iy = ((gv.y + 1.f) * (float)H - 1.f) / 2.f;
  s.x0 = (int)floorf(s.ix);
  s.y0 = (int)floorf(s.iy);
  return s;
}

// one thread per output pixel of one copy, its 3 channels
__global__ void __launch_bounds__(256) aug_fwd_kernel(const float* __restrict__ img, const float* __restrict__ grid,
                                                      float* __restrict__ out, int64_t total, int K, int H, int W,
                                                      int Ho, int Wo, float shift) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t HWo = (int64_t)Ho * Wo;
  const int64_t j = i / HWo;                     // copy b*K + k
  const int pix = (int)(i - j * HWo);
  const int b = (int)(j / K);
  const Samp s = samp_at(grid + i * 2, W, H);
  const float fx = (float)s.x0, fy = (float)s.y0;
  const float nw = (fx + 1.f - s.ix) * (fy + 1.f - s.iy), ne = (s.ix - fx) * (fy + 1.f - s.iy);
  const float sw = (fx + 1.f - s.ix) * (s.iy - fy), se = (s.ix - fx) * (s.iy - fy);
  const float* im = img + (int64_t)b * H * W * 3;
  float acc[3] = {0.f, 0.f, 0.f};
  const int cx[4] = {s.x0, s.x0 + 1, s.x0, s.x0 + 1}, cy[4] = {s.y0, s.y0, s.y0 + 1, s.y0 + 1};
  const float wt[4] = {nw, ne, sw, se};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bool in = cx[q] >= 0 && cx[q] < W && cy[q] >= 0 && cy[q] < H;
    const int64_t o = ((int64_t)min(max(cy[q], 0), H - 1) * W + min(max(cx[q], 0), W - 1)) * 3;
    const float v0 = im[o] - shift, v1 = im[o + 1] - shift, v2 = im[o + 2] - shift;
    acc[0] = in ? acc[0] + v0 * wt[q] : acc[0];
    acc[1] = in ? acc[1] + v1 * wt[q] : acc[1];
    acc[2] = in ? acc[2] + v2 * wt[q] : acc[2];
  }
  float* op = out + j * 3 * HWo + pix;
#pragma unroll
  for (int c = 0; c < 3; ++c) op[c * HWo] = acc[c] + shift;
}

// F.affine_grid(theta, [N, C, H, W], align_corners=False): ATen's base grid (linspace(-1, 1, n) scaled
// by (n - 1) / n; linspace's two-sided form: start + step i below the middle, end - step (n - 1 - i)
// above) times theta^T, the three products accumulated x, y, translation
__device__ __forceinline__ float affine_base(int i, int n) {
  if (n == 1) return 0.f;   // linspace(-1, 1, 1) = [-1], times 0 / 1
  const float step = 2.f / (float)(n - 1);
  const float v = i < n / 2 ? -1.f + step * (float)i : 1.f - step * (float)(n - 1 - i);
  return v * (float)(n - 1) / (float)n;
}
__global__ void __launch_bounds__(256) affine_grid_kernel(const float* __restrict__ theta, int64_t total, int H, int W,
                                                          float* __restrict__ grid) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t HW = (int64_t)H * W;
  const int64_t n = i / HW;
  const int pix = (int)(i - n * HW);
  const int y = pix / W, x = pix - y * W;
  const float bx = affine_base(x, W), by = affine_base(y, H);
  const float* t = theta + n * 6;
  float2 g;
  g.x = fmaf(1.f, t[2], fmaf(by, t[1], bx * t[0]));
  g.y = fmaf(1.f, t[5], fmaf(by, t[4], bx * t[3]));
  reinterpret_cast<float2*>(grid)[i] = g;
}

// Adjoint, gathered (no atomics): a workgroup takes 64 consecutive input pixels (b, Y, X), one per
// lane, and its four waves the copies k = wave, wave + 4, ...; for each copy the output pixels whose
// sample has (Y, X) as a corner lie in the preimage of the 2x2 box around (Y, X) under the copy's
// affine map (read off the grid itself: its value at (0,0), (0,1), (1,0)), enumerated over that
// preimage's bounding box + 1 and tested with the forward's exact arithmetic; the four waves' sums
// are combined in LDS in wave order.  The lanes of a wave hold neighbouring pixels of ONE copy, so an
// enumeration step's grid and gradient reads are neighbouring addresses (round 4 had 16 lanes per
// pixel on 16 copies: every read a separate line, 110 us per vgg step).
__global__ void __launch_bounds__(256) aug_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ grid,
                                                      float* __restrict__ gimg, int64_t total, int K, int H, int W,
                                                      int Ho, int Wo) {
  __shared__ float part[3][4][64];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + l;   // input pixel
  const bool live = i < total;
  const int64_t ic = live ? i : total - 1;
  const int64_t HW = (int64_t)H * W, HWo = (int64_t)Ho * Wo;
  const int b = (int)(ic / HW);
  const int pix = (int)(ic - (int64_t)b * HW);
  const int Y = pix / W, X = pix - Y * W;
  float acc[3] = {0.f, 0.f, 0.f};
  for (int k = wv; k < K; k += 4) {
    const int64_t j = (int64_t)b * K + k;
    const float* gj = grid + j * HWo * 2;
    // source position as an affine function of the output pixel, s(x, y) = s00 + x dx + y dy,
    // its slopes read across the whole grid (the grid's rounding ~1e-6 px then moves them by
    // ~1e-8 per pixel)
    const Samp s00 = samp_at(gj, W, H), s01 = samp_at(gj + 2 * (Wo - 1), W, H),
               s10 = samp_at(gj + 2 * (int64_t)(Ho - 1) * Wo, W, H);
    const float ax = Wo > 1 ? (s01.ix - s00.ix) / (float)(Wo - 1) : 1.f;
    const float ay = Wo > 1 ? (s01.iy - s00.iy) / (float)(Wo - 1) : 0.f;
    const float bx = Ho > 1 ? (s10.ix - s00.ix) / (float)(Ho - 1) : 0.f;
    const float by = Ho > 1 ? (s10.iy - s00.iy) / (float)(Ho - 1) : 1.f;
    const float det = ax * by - bx * ay;
    if (!(fabsf(det) > 1e-12f)) continue;        // degenerate map (never drawn: scale > 0)
    const float i00 = by / det, i01 = -bx / det, i10 = -ay / det, i11 = ax / det;
    // the samples with corner (X, Y) have ix in [X-1, X+1), iy in [Y-1, Y+1): the preimage of
    // that box is centred on the preimage of (X, Y), half extent |inverse| (1, 1) (+0.05 px)
    const float px = (float)X - s00.ix, py = (float)Y - s00.iy;
    const float cx = i00 * px + i01 * py, cy = i10 * px + i11 * py;
    const float ex = fabsf(i00) + fabsf(i01) + 0.05f, ey = fabsf(i10) + fabsf(i11) + 0.05f;
    const int xlo = max((int)floorf(cx - ex), 0), xhi = min((int)ceilf(cx + ex), Wo - 1);
    const int ylo = max((int)floorf(cy - ey), 0), yhi = min((int)ceilf(cy + ey), Ho - 1);
    const float* go = gout + j * 3 * HWo;
    for (int y = ylo; y <= yhi; ++y) {
      // four box columns per pass: their grid reads issued together (the walk is a chain of dependent
      // grid read -> test -> gradient read; one column at a time exposes each read's latency)
      for (int x = xlo; x <= xhi; x += 4) {
        Samp s[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) s[u] = samp_at(gj + ((int64_t)y * Wo + min(x + u, xhi)) * 2, W, H);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t o = (int64_t)y * Wo + x + u;
          const int dxc = X - s[u].x0, dyc = Y - s[u].y0;
          if (x + u > xhi || dxc < 0 || dxc > 1 || dyc < 0 || dyc > 1) continue;
          const float fx = (float)s[u].x0, fy = (float)s[u].y0;
          const float wxv = dxc ? (s[u].ix - fx) : (fx + 1.f - s[u].ix);
          const float wyv = dyc ? (s[u].iy - fy) : (fy + 1.f - s[u].iy);
          const float w = wxv * wyv;
          acc[0] += w * go[o];
          acc[1] += w * go[HWo + o];
          acc[2] += w * go[2 * HWo + o];
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) part[c][wv][l] = acc[c];
  // (wait states behind the LDS stores before their data registers are rewritten: the wide-store
  //  data hazard nfi_common.h's lds_st guards, checked by scripts/isa_lint.py)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();
  // 64 pixels x 3 channels, contiguous in gimg [B][H][W][3]
  const int t = threadIdx.x;
  if (t < 192) {
    const int p = t / 3, c = t - 3 * p;
    const int64_t o = (int64_t)blockIdx.x * 64 + p;
    if (o < total) gimg[o * 3 + c] = (part[c][0][p] + part[c][1][p]) + (part[c][2][p] + part[c][3][p]);
  }
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }


// ---------------------------------------------------------------------------------------
// AttentionMapper conditional norm layer (generator.py:42-60, 160-178):
//   x = leaky_relu(beta + gamma1 * layer_norm(h), 0.2),  layer_norm without affine, eps 1e-5
// one workgroup per row (C <= 1024 channels, 256 threads x 4), mean / rstd saved for the backward:
//   gz = gx * slope(z); d beta = gz; d gamma1 = gz * y; gy = gz * gamma1;
//   d h = rstd * (gy - mean(gy) - y * mean(gy * y))   (ATen's layer_norm backward)
// (the mapper's 4 norms: 3 ATen kernels forward and ~6 backward each -> 1 + 1)
// ---------------------------------------------------------------------------------------
constexpr int CLN_PER = 4;   // channels per thread (C <= 1024)
__device__ __forceinline__ void block_sum2(float& a, float& b) {
  __shared__ float red[2][4];
  a = wave_sum(a);
  b = wave_sum(b);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
    // (wait states behind the paired LDS store before its data registers are rewritten: the
    //  wide-store data hazard nfi_common.h's lds_st guards, checked by scripts/isa_lint.py)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  a = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  b = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
}

__global__ void __launch_bounds__(256) cln_act_fwd_kernel(const float* __restrict__ h, const float* __restrict__ g1,
                                                          const float* __restrict__ be, int ld, int C,
                                                          float* __restrict__ x, float* __restrict__ stats) {
  const int row = blockIdx.x;
  const float* hr = h + (long long)row * C;
  float v[CLN_PER], s1 = 0.f, s0 = 0.f;
#pragma unroll
  for (int k = 0; k < CLN_PER; ++k) {
    const int c = threadIdx.x + 256 * k;
    v[k] = c < C ? hr[c] : 0.f;
    s1 += v[k];
  }
  block_sum2(s1, s0);
  const float mean = s1 / (float)C;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < CLN_PER; ++k) {
    const int c = threadIdx.x + 256 * k;
    const float d = c < C ? v[k] - mean : 0.f;
    s2 += d * d;
  }
  s0 = 0.f;
  block_sum2(s2, s0);
  const float rstd = rsqrtf(s2 / (float)C + 1e-5f);
#pragma unroll
  for (int k = 0; k < CLN_PER; ++k) {
    const int c = threadIdx.x + 256 * k;
    if (c < C) {
      const float z = be[(long long)row * ld + c] + g1[(long long)row * ld + c] * ((v[k] - mean) * rstd);
      x[(long long)row * C + c] = z > 0.f ? z : 0.2f * z;
    }
  }
  if (threadIdx.x == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = rstd;
  }
}

__global__ void __launch_bounds__(256) cln_act_bwd_kernel(const float* __restrict__ gx, const float* __restrict__ h,
                                                          const float* __restrict__ g1, const float* __restrict__ be,
                                                          int ld, int C, const float* __restrict__ stats,
                                                          float* __restrict__ dh, float* __restrict__ dg1,
                                                          float* __restrict__ dbe) {
  const int row = blockIdx.x;
  const float mean = stats[2 * row], rstd = stats[2 * row + 1];
  float y[CLN_PER], gy[CLN_PER], a = 0.f, b = 0.f;
#pragma unroll
  for (int k = 0; k < CLN_PER; ++k) {
    const int c = threadIdx.x + 256 * k;
    y[k] = gy[k] = 0.f;
    if (c < C) {
      const long long i = (long long)row * C + c, ic = (long long)row * ld + c;
      y[k] = (h[i] - mean) * rstd;
      const float gam = g1[ic];
      const float z = be[ic] + gam * y[k];
      const float gz = z > 0.f ? gx[i] : 0.2f * gx[i];
      dbe[i] = gz;
      dg1[i] = gz * y[k];
      gy[k] = gz * gam;
      a += gy[k];
      b += gy[k] * y[k];
    }
  }
  block_sum2(a, b);
  const float ma = a / (float)C, mb = b / (float)C;
#pragma unroll
  for (int k = 0; k < CLN_PER; ++k) {
    const int c = threadIdx.x + 256 * k;
    if (c < C) dh[(long long)row * C + c] = rstd * (gy[k] - ma - y[k] * mb);
  }
}

}  // namespace syn
}  // namespace nfi

using namespace nfi::syn;

extern "C" {

int32_t nfi_syn_act_forward(const float* o, const float* d, const float* bias, float* y, int32_t P,
                            int32_t C, int32_t HW, float gain, void* stream) {
  NFI_REQUIRE(o && d && bias && y, "syn_act_forward: null pointer");
  NFI_REQUIRE(P > 0 && C > 0 && P % C == 0 && HW > 0 && HW % 4 == 0, "syn_act_forward: bad shape");
  const int64_t n4 = (int64_t)P * (HW / 4);
  act_fwd_kernel<<<blocks(n4), 256, 0, (hipStream_t)stream>>>((const float4*)o, d, bias, (float4*)y,
                                                               n4, C, HW / 4, gain);
  NFI_CHECK_LAUNCH("act_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_act_backward(const float* g, const float* o, const float* d, const float* bias,
                             float* go, float* dd, int32_t P, int32_t C, int32_t HW, float gain,
                             void* stream) {
  NFI_REQUIRE(g && o && d && bias && go && dd, "syn_act_backward: null pointer");
  NFI_REQUIRE(P > 0 && C > 0 && P % C == 0 && HW > 0 && HW % 4 == 0, "syn_act_backward: bad shape");
  hipStream_t s = (hipStream_t)stream;
  const int HW4 = HW / 4;
  if (HW4 > RED_CHUNK4 && hipMemsetAsync(dd, 0, sizeof(float) * P, s) != hipSuccess) {
    nfi::set_error("syn_act_backward: memset failed");
    return NFI_ELAUNCH;
  }
  act_bwd_kernel<<<dim3((HW4 + RED_CHUNK4 - 1) / RED_CHUNK4, P), 256, 0, s>>>(
      (const float4*)g, (const float4*)o, d, bias, (float4*)go, dd, C, HW4, gain);
  NFI_CHECK_LAUNCH("act_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_fir_up_act_forward(const float* t, const float* d, const float* bias, float* o,
                                   float* y, int32_t P, int32_t C, int32_t n, float gain,
                                   void* stream) {
  NFI_REQUIRE(t && d && bias && o && y, "syn_fir_up_act_forward: null pointer");
  NFI_REQUIRE(P > 0 && C > 0 && P % C == 0 && n >= 2 && n % 2 == 0, "syn_fir_up_act_forward: bad shape");
  const int64_t n4 = (int64_t)P * (2 * n) * (2 * n) / 4;
  fir_up_act_kernel<<<blocks(n4), 256, 0, (hipStream_t)stream>>>(t, d, bias, (float4*)o, (float4*)y,
                                                                  n4, C, n, gain);
  NFI_CHECK_LAUNCH("fir_up_act_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_conv_scatter(const float* P, float* t, int32_t B, int32_t C, int32_t n, void* stream) {
  NFI_REQUIRE(P && t, "syn_up_conv_scatter: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && n >= 1, "syn_up_conv_scatter: bad shape");
  const int64_t total = (int64_t)B * C * (2 * n + 1) * (2 * n + 1);
  tap_scatter_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(P, t, total, C, n);
  NFI_CHECK_LAUNCH("tap_scatter_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_conv_fir_act_forward(const float* P, const float* d, const float* bias, float* o, float* y,
                                        int32_t B, int32_t C, int32_t n, float gain, void* stream) {
  NFI_REQUIRE(P && d && bias && o && y, "syn_up_conv_fir_act_forward: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && n > 0 && (2 * n) % UF_TX == 0, "syn_up_conv_fir_act_forward: bad shape");
  const int W2 = 2 * n;
  up_fir_act_kernel<<<dim3((unsigned)((W2 / UF_TY) * (W2 / UF_TX)), (unsigned)(B * C)), 256, 0,
                      (hipStream_t)stream>>>(P, d, bias, (float4*)o, (float4*)y, C, n, gain);
  NFI_CHECK_LAUNCH("up_fir_act_kernel");
  return NFI_OK;
}

static int32_t up_conv_act_backward(const float* g, const float* o, const float* d, const float* bias, float* dP,
                                   float* dd, int32_t B, int32_t C, int32_t n, float gain, uint32_t* vmax, void* stream) {
  NFI_REQUIRE(g && o && d && bias && dP && dd, "syn_up_conv_act_backward: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && n > 0 && n % UB_TX == 0, "syn_up_conv_act_backward: bad shape");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(dd, 0, sizeof(float) * B * C, st) != hipSuccess) {
    nfi::set_error("syn_up_conv_act_backward: memset failed");
    return NFI_ELAUNCH;
  }
  up_bwd_fused_kernel<<<dim3((unsigned)((n / UB_TY) * (n / UB_TX)), (unsigned)(B * C)), 256, 0, st>>>(
      g, o, d, bias, dP, dd, C, n, gain, (unsigned*)vmax);
  NFI_CHECK_LAUNCH("up_bwd_fused_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_conv_act_backward(const float* g, const float* o, const float* d, const float* bias, float* dP,
                                     float* dd, int32_t B, int32_t C, int32_t n, float gain, void* stream) {
  return up_conv_act_backward(g, o, d, bias, dP, dd, B, C, n, gain, nullptr, stream);
}

int32_t nfi_syn_up_conv_act_backward_max(const float* g, const float* o, const float* d, const float* bias, float* dP,
                                         float* dd, uint32_t* vmax, int32_t B, int32_t C, int32_t n, float gain,
                                         void* stream) {
  NFI_REQUIRE(vmax, "syn_up_conv_act_backward_max: null vmax");
  return up_conv_act_backward(g, o, d, bias, dP, dd, B, C, n, gain, vmax, stream);
}

int32_t nfi_syn_up_conv_gather(const float* gt, float* dP, int32_t B, int32_t C, int32_t n, void* stream) {
  NFI_REQUIRE(gt && dP, "syn_up_conv_gather: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && n >= 1, "syn_up_conv_gather: bad shape");
  const int64_t total = (int64_t)B * C * n * n;
  tap_gather_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(gt, dP, total, C, n);
  NFI_CHECK_LAUNCH("tap_gather_kernel");
  return NFI_OK;
}

int32_t nfi_syn_fir_up_backward(const float* go, float* gt, int32_t P, int32_t n, void* stream) {
  NFI_REQUIRE(go && gt && P > 0 && n >= 1, "syn_fir_up_backward: bad args");
  const int64_t total = (int64_t)P * (2 * n + 1) * (2 * n + 1);
  fir_up_bwd_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(go, gt, total, n);
  NFI_CHECK_LAUNCH("fir_up_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_add_forward(const float* img, const float* c, const float* bias, float* out,
                               int32_t P, int32_t C, int32_t n, void* stream) {
  NFI_REQUIRE(c && bias && out, "syn_up_add_forward: null pointer");
  NFI_REQUIRE(P > 0 && C > 0 && P % C == 0 && n >= 2 && n % 2 == 0, "syn_up_add_forward: bad shape");
  const int64_t n4 = (int64_t)P * (2 * n) * (2 * n) / 4;
  up_add_kernel<<<blocks(n4), 256, 0, (hipStream_t)stream>>>(img, (const float4*)c, bias,
                                                              (float4*)out, n4, C, n);
  NFI_CHECK_LAUNCH("up_add_kernel");
  return NFI_OK;
}

static int str4_of(const int64_t* s, Str4& o) {
  // float strides (b, q, t) -> float4 units; every one a multiple of 4 floats
  if (s[0] % 4 || s[1] % 4 || s[2] % 4) return 0;
  o = Str4{s[0] / 4, s[1] / 4, s[2] / 4};
  return 1;
}

int32_t nfi_syn_up_add_forward_strided(const float* img, const int64_t* img_strides, const float* c,
                                       const int64_t* c_strides, const float* bias, float* out,
                                       const int64_t* out_strides, int32_t B, int32_t C, int32_t n, void* stream) {
  NFI_REQUIRE(c && bias && out && c_strides && out_strides && (!img || img_strides),
              "syn_up_add_forward_strided: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && C % 4 == 0 && n >= 1, "syn_up_add_forward_strided: bad shape");
  Str4 si{0, 0, 0}, sc, so;
  NFI_REQUIRE((!img || str4_of(img_strides, si)) && str4_of(c_strides, sc) && str4_of(out_strides, so),
              "syn_up_add_forward_strided: strides must be multiples of 4 floats");
  const int64_t total4 = (int64_t)B * (2 * n) * (2 * n) * (C / 4);
  up_add_str_kernel<<<blocks(total4), 256, 0, (hipStream_t)stream>>>(
      (const float4*)img, si, (const float4*)c, sc, (const float4*)bias, (float4*)out, so, total4, C / 4, n);
  NFI_CHECK_LAUNCH("up_add_str_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_backward_strided(const float* g, const int64_t* g_strides, float* gimg, const int64_t* gimg_strides,
                                    int32_t B, int32_t C, int32_t n, void* stream) {
  NFI_REQUIRE(g && gimg && g_strides && gimg_strides && B > 0 && C > 0 && C % 4 == 0 && n >= 1,
              "syn_up_backward_strided: bad args");
  Str4 sg, sr;
  NFI_REQUIRE(str4_of(g_strides, sg) && str4_of(gimg_strides, sr),
              "syn_up_backward_strided: strides must be multiples of 4 floats");
  const int64_t total4 = (int64_t)B * n * n * (C / 4);
  up_bwd_str_kernel<<<blocks(total4), 256, 0, (hipStream_t)stream>>>((const float4*)g, sg, (float4*)gimg, sr,
                                                                    total4, C / 4, n);
  NFI_CHECK_LAUNCH("up_bwd_str_kernel");
  return NFI_OK;
}

int32_t nfi_syn_up_backward(const float* g, float* gimg, int32_t P, int32_t n, void* stream) {
  NFI_REQUIRE(g && gimg && P > 0 && n >= 1, "syn_up_backward: bad args");
  const int64_t total = (int64_t)P * n * n;
  up_bwd_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(g, gimg, total, n);
  NFI_CHECK_LAUNCH("up_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_scale_backward(const float* g, const float* x, const float* s, float* gx, float* ds,
                               int32_t P, int32_t HW, void* stream) {
  NFI_REQUIRE(g && x && s && ds, "syn_scale_backward: null pointer");
  NFI_REQUIRE(P > 0 && HW > 0 && HW % 4 == 0, "syn_scale_backward: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const int HW4 = HW / 4;
  if (HW4 > RED_CHUNK4 && hipMemsetAsync(ds, 0, sizeof(float) * P, st) != hipSuccess) {
    nfi::set_error("syn_scale_backward: memset failed");
    return NFI_ELAUNCH;
  }
  scale_bwd_kernel<<<dim3((HW4 + RED_CHUNK4 - 1) / RED_CHUNK4, P), 256, 0, st>>>(
      (const float4*)g, (const float4*)x, s, (float4*)gx, ds, HW4);
  NFI_CHECK_LAUNCH("scale_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_lpips_head_forward(const float* f0, const float* f1, const float* w, float* out,
                               float* inv0, float* inv1, int32_t N, int32_t C, int32_t HW,
                               void* stream) {
  NFI_REQUIRE(f0 && f1 && w && out && inv0 && inv1, "lpips_head_forward: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && HW > 0, "lpips_head_forward: bad shape");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(out, 0, sizeof(float) * N, st) != hipSuccess) {
    nfi::set_error("lpips_head_forward: memset failed");
    return NFI_ELAUNCH;
  }
  const unsigned pb = (unsigned)(((int64_t)N * HW + 63) / 64);
  switch (C) {
    case 64: lpips_fwd_regs_kernel<4, 16><<<pb, 256, 0, st>>>(f0, f1, w, out, inv0, inv1, N, HW); break;
    case 128: lpips_fwd_regs_kernel<8, 16><<<pb, 512, 0, st>>>(f0, f1, w, out, inv0, inv1, N, HW); break;
    case 256: lpips_fwd_regs_kernel<16, 16><<<pb, 1024, 0, st>>>(f0, f1, w, out, inv0, inv1, N, HW); break;
    case 512: lpips_fwd_regs_kernel<16, 32><<<pb, 1024, 0, st>>>(f0, f1, w, out, inv0, inv1, N, HW); break;
    default: lpips_fwd_kernel<<<blocks((int64_t)N * HW), 256, 0, st>>>(f0, f1, w, out, inv0, inv1, N, C, HW);
  }
  NFI_CHECK_LAUNCH("lpips_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_lpips_head_backward(const float* g, const float* f0, const float* f1, const float* w,
                                const float* inv0, const float* inv1, float* gf0, int32_t N,
                                int32_t C, int32_t HW, void* stream) {
  NFI_REQUIRE(g && f0 && f1 && w && inv0 && inv1 && gf0, "lpips_head_backward: null pointer");
  NFI_REQUIRE(N > 0 && C > 0 && HW > 0, "lpips_head_backward: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const unsigned pb = (unsigned)(((int64_t)N * HW + 63) / 64);
  switch (C) {
    case 64: lpips_bwd_regs_kernel<4, 16><<<pb, 256, 0, st>>>(g, f0, f1, w, inv0, inv1, gf0, N, HW); break;
    case 128: lpips_bwd_regs_kernel<8, 16><<<pb, 512, 0, st>>>(g, f0, f1, w, inv0, inv1, gf0, N, HW); break;
    case 256: lpips_bwd_regs_kernel<16, 16><<<pb, 1024, 0, st>>>(g, f0, f1, w, inv0, inv1, gf0, N, HW); break;
    case 512: lpips_bwd_regs_kernel<16, 32><<<pb, 1024, 0, st>>>(g, f0, f1, w, inv0, inv1, gf0, N, HW); break;
    default: lpips_bwd_kernel<<<blocks((int64_t)N * HW), 256, 0, st>>>(g, f0, f1, w, inv0, inv1, gf0, N, C, HW);
  }
  NFI_CHECK_LAUNCH("lpips_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_vgg_first_forward_max(const float* x, const float* nshift, const float* nscale, const float* w,
                                  const float* bias, float* y, uint32_t* ymax, int32_t N, int32_t Co, int32_t H, int32_t W,
                                  void* stream) {
  NFI_REQUIRE((nshift == nullptr) == (nscale == nullptr), "vgg_first_forward: shift and scale go together");
  NFI_REQUIRE(x && w && bias && y, "vgg_first_forward: null pointer");
  NFI_REQUIRE(N > 0 && Co > 0 && H > 0 && W > 0 && W % 4 == 0, "vgg_first_forward: bad shape");
  const int64_t total = (int64_t)N * H * (W / 4);
  vgg_first_fwd_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(x, w, bias, (float4*)y, total, Co, H, W,
                                                                       (unsigned*)ymax, nshift, nscale);
  NFI_CHECK_LAUNCH("vgg_first_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_vgg_first_forward(const float* x, const float* w, const float* bias, float* y, int32_t N, int32_t Co,
                              int32_t H, int32_t W, void* stream) {
  return nfi_vgg_first_forward_max(x, nullptr, nullptr, w, bias, y, nullptr, N, Co, H, W, stream);
}

int32_t nfi_vgg_first_backward_scaled(const float* gy, const float* y, const float* w, const float* nscale, float* gx,
                                      int32_t N, int32_t Co,
                               int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(gy && y && w && gx, "vgg_first_backward: null pointer");
  NFI_REQUIRE(N > 0 && Co > 0 && H % VF_TY == 0 && W % VF_TX == 0, "vgg_first_backward: bad shape");
  vgg_first_bwd_kernel<<<dim3((unsigned)((H / VF_TY) * (W / VF_TX)), (unsigned)N), 256, 0, (hipStream_t)stream>>>(
      gy, y, w, gx, Co, H, W, nscale);
  NFI_CHECK_LAUNCH("vgg_first_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_vgg_first_backward(const float* gy, const float* y, const float* w, float* gx, int32_t N, int32_t Co,
                               int32_t H, int32_t W, void* stream) {
  return nfi_vgg_first_backward_scaled(gy, y, w, nullptr, gx, N, Co, H, W, stream);
}

int32_t nfi_vgg_bias_relu_forward(const float* x, const float* bias, float* y, float* pooled,
                                  int32_t P, int32_t C, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(x && bias && y, "vgg_bias_relu_forward: null pointer");
  NFI_REQUIRE(P > 0 && C > 0 && P % C == 0 && H > 0 && W > 0 && W % 4 == 0,
              "vgg_bias_relu_forward: bad shape (W % 4 == 0 required)");
  NFI_REQUIRE(!pooled || H % 2 == 0, "vgg_bias_relu_forward: pooling needs an even height");
  hipStream_t st = (hipStream_t)stream;
  if (pooled) {
    const int64_t np = (int64_t)P * (H / 2) * (W / 4);
    vgg_bias_relu_pool_kernel<<<blocks(np), 256, 0, st>>>(x, bias, y, pooled, np, C, H, W);
    NFI_CHECK_LAUNCH("vgg_bias_relu_pool_kernel");
  } else {
    const int64_t n4 = (int64_t)P * H * W / 4;
    vgg_bias_relu_kernel<<<blocks(n4), 256, 0, st>>>((const float4*)x, bias, (float4*)y, n4, C, H * W / 4);
    NFI_CHECK_LAUNCH("vgg_bias_relu_kernel");
  }
  return NFI_OK;
}

int32_t nfi_vgg_relu_backward_max(const float* gy, const float* gpooled, const float* y, float* gx, uint32_t* gmax,
                                  int32_t P, int32_t C, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(y && gx && gpooled && gmax && C > 0 && P % C == 0, "vgg_relu_backward_max: bad arguments");
  NFI_REQUIRE(P > 0 && H > 0 && W > 0 && W % 4 == 0 && H % 2 == 0, "vgg_relu_backward_max: bad shape");
  const int64_t np = (int64_t)P * (H / 2) * (W / 4);
  vgg_relu_pool_bwd_kernel<<<blocks(np), 256, 0, (hipStream_t)stream>>>(gy, gpooled, y, gx, np, H, W, (unsigned*)gmax, C);
  NFI_CHECK_LAUNCH("vgg_relu_pool_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_vgg_relu_backward(const float* gy, const float* gpooled, const float* y, float* gx,
                              int32_t P, int32_t H, int32_t W, void* stream) {
  NFI_REQUIRE(y && gx && (gy || gpooled), "vgg_relu_backward: null pointer");
  NFI_REQUIRE(P > 0 && H > 0 && W > 0 && W % 4 == 0, "vgg_relu_backward: bad shape (W % 4 == 0 required)");
  NFI_REQUIRE(!gpooled || H % 2 == 0, "vgg_relu_backward: pooling needs an even height");
  hipStream_t st = (hipStream_t)stream;
  if (gpooled) {
    const int64_t np = (int64_t)P * (H / 2) * (W / 4);
    vgg_relu_pool_bwd_kernel<<<blocks(np), 256, 0, st>>>(gy, gpooled, y, gx, np, H, W, nullptr, 1);
    NFI_CHECK_LAUNCH("vgg_relu_pool_bwd_kernel");
  } else {
    const int64_t n4 = (int64_t)P * H * W / 4;
    vgg_relu_bwd_kernel<<<blocks(n4), 256, 0, st>>>((const float4*)gy, (const float4*)y, (float4*)gx, n4);
    NFI_CHECK_LAUNCH("vgg_relu_bwd_kernel");
  }
  return NFI_OK;
}

int32_t nfi_aug_sample_forward(const float* img, const float* grid, float* out, int32_t B, int32_t K, int32_t H,
                               int32_t W, int32_t Ho, int32_t Wo, float shift, void* stream) {
  NFI_REQUIRE(img && grid && out, "aug_sample_forward: null pointer");
  NFI_REQUIRE(B > 0 && K > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, "aug_sample_forward: bad shape");
  const int64_t total = (int64_t)B * K * Ho * Wo;
  aug_fwd_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(img, grid, out, total, K, H, W, Ho, Wo, shift);
  NFI_CHECK_LAUNCH("aug_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_aug_affine_grid(const float* theta, int32_t N, int32_t H, int32_t W, float* grid, void* stream) {
  NFI_REQUIRE(theta && grid, "aug_affine_grid: null pointer");
  NFI_REQUIRE(N > 0 && H > 0 && W > 0, "aug_affine_grid: bad shape N=%d H=%d W=%d", N, H, W);
  NFI_REQUIRE(((uintptr_t)grid & 7) == 0, "aug_affine_grid: grid must be 8-B aligned");
  const int64_t total = (int64_t)N * H * W;
  affine_grid_kernel<<<blocks(total), 256, 0, (hipStream_t)stream>>>(theta, total, H, W, grid);
  NFI_CHECK_LAUNCH("affine_grid_kernel");
  return NFI_OK;
}

int32_t nfi_aug_sample_backward(const float* gout, const float* grid, float* gimg, int32_t B, int32_t K, int32_t H,
                                int32_t W, int32_t Ho, int32_t Wo, void* stream) {
  NFI_REQUIRE(gout && grid && gimg, "aug_sample_backward: null pointer");
  NFI_REQUIRE(B > 0 && K > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, "aug_sample_backward: bad shape");
  const int64_t total = (int64_t)B * H * W;
  aug_bwd_kernel<<<(unsigned)((total + 63) / 64), 256, 0, (hipStream_t)stream>>>(gout, grid, gimg, total, K, H, W, Ho, Wo);
  NFI_CHECK_LAUNCH("aug_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_cond_norm_act_forward(const float* h, const float* gamma1, const float* beta, int32_t B, int32_t C,
                                      int32_t ld, float* x, float* stats, void* stream) {
  NFI_REQUIRE(h && gamma1 && beta && x && stats, "syn_cond_norm_act_forward: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && C <= 256 * CLN_PER && ld >= C, "syn_cond_norm_act_forward: bad shape B=%d C=%d ld=%d",
              B, C, ld);
  cln_act_fwd_kernel<<<B, 256, 0, (hipStream_t)stream>>>(h, gamma1, beta, ld, C, x, stats);
  NFI_CHECK_LAUNCH("cln_act_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_syn_cond_norm_act_backward(const float* gx, const float* h, const float* gamma1, const float* beta,
                                       const float* stats, int32_t B, int32_t C, int32_t ld, float* dh,
                                       float* dgamma1, float* dbeta, void* stream) {
  NFI_REQUIRE(gx && h && gamma1 && beta && stats && dh && dgamma1 && dbeta,
              "syn_cond_norm_act_backward: null pointer");
  NFI_REQUIRE(B > 0 && C > 0 && C <= 256 * CLN_PER && ld >= C, "syn_cond_norm_act_backward: bad shape B=%d C=%d ld=%d",
              B, C, ld);
  cln_act_bwd_kernel<<<B, 256, 0, (hipStream_t)stream>>>(gx, h, gamma1, beta, ld, C, stats, dh, dgamma1, dbeta);
  NFI_CHECK_LAUNCH("cln_act_bwd_kernel");
  return NFI_OK;
}

}  // extern "C"
