// Ray bundle, near/far planes, their backward, per-image reductions, decoder packing and
// plane layout conversion.  gfx950 (MI355X).  All kernels are simple per-element
// HBM-streaming kernels; the hot path is nfi_render.hip.
#include <string.h>
#include <cmath>
#include <string>

#include "nfi_common.h"
#include "nfi_host.h"

namespace nfi {

static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

// ---------------------------------------------------------------------------------------
// Ray bundle (nerf_utils.py:28-93) + F.normalize (run.py:196) + slab test (nerf_utils.py:227-275)
// ---------------------------------------------------------------------------------------


// Camera-space quantities of pixel (x, y) of image b, exactly as nerf_utils.py computes them.
__device__ __forceinline__ void pixel_coords(const nfi_camera& c, int b, int x, int y, float& ii,
                                             float& jj) {
  ii = fdiv((float)x, (float)c.W);   // arange(W)/W  (meshgrid indexing='xy': ii varies along W)
  jj = fdiv((float)y, (float)c.H);
  if (c.focal) {
    if (c.center) {
      ii = fsub(fsub(ii, fmul(0.5f, fsub(fmul(2.f, c.center[b * 2 + 0]), 1.f))), 0.5f);
      jj = fsub(fsub(jj, fmul(0.5f, fsub(fmul(2.f, c.center[b * 2 + 1]), 1.f))), 0.5f);
    } else {
      ii = fsub(ii, 0.5f);
      jj = fsub(jj, 0.5f);
    }
    if (c.bbox) {
      const float* bb = c.bbox + b * 4;   // bbox[b][i][j] = bb[i*2+j]
      ii = fmul(fadd(fmul(bb[2], fadd(ii, 0.5f)), bb[0]), 0.5f);
      jj = fmul(-fadd(fmul(bb[3], fadd(-jj, 0.5f)), bb[1]), 0.5f);
    }
  } else {
    ii = fmul(fsub(ii, 0.5f), 2.f);
    jj = fmul(fsub(jj, 0.5f), 2.f);
    if (c.bbox) {
      const float* bb = c.bbox + b * 4;
      ii = fadd(fmul(bb[2], fadd(fdiv(ii, 2.f), 0.5f)), bb[0]);
      jj = -fadd(fmul(bb[3], fadd(fdiv(-jj, 2.f), 0.5f)), bb[1]);
    }
  }
}

// sum_k v[k] * M[i][k] as torch.sum(v[...,None,:] * M, -1) on CPU: rounded products, left to right
__device__ __forceinline__ float rowdot3(const float v[3], const float* __restrict__ Mi) {
  return fadd(fadd(fmul(v[0], Mi[0]), fmul(v[1], Mi[1])), fmul(v[2], Mi[2]));
}

__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fdecode(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Slab test of one ray against [-sr, sr]^3 as nerf_utils.py:235-258 evaluates it (invdir = 1/d,
// the bound picked by the sign of invdir, products of rounded differences); returns the hit flag.
__device__ __forceinline__ bool slab_test(const float o[3], const float d[3], float sr, float& nr, float& fr) {
  float tmin[3], tmax[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float inv = fdiv(1.f, d[i]);
    const bool neg = inv < 0.f;
    tmin[i] = fmul(fsub(neg ? sr : -sr, o[i]), inv);
    tmax[i] = fmul(fsub(neg ? -sr : sr, o[i]), inv);
  }
  bool hit = !((tmin[0] > tmax[1]) || (tmin[1] > tmax[0]));
  nr = fmaxf(tmin[0], tmin[1]);
  fr = fminf(tmax[0], tmax[1]);
  hit = hit && !((nr > tmax[2]) || (tmin[2] > fr));
  nr = fmaxf(nr, tmin[2]);
  fr = fminf(fr, tmax[2]);
  return hit;
}

// min near / max far over the hits of a 256-ray block as order-preserving keys into part[2 block]
// (combined by rays_fix_kernel: no contended atomics on one address), nerf_utils.py:260-261
__device__ __forceinline__ void block_hit_range(bool hit, float nr, float fr, uint32_t* __restrict__ part) {
  __shared__ uint32_t red[2][4];
  uint32_t kmin = hit ? fkey(nr) : 0xFFFFFFFFu;
  uint32_t kmax = hit ? fkey(fr) : 0u;
  for (int o = 32; o > 0; o >>= 1) {
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = kmin;
    red[1][threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3]));
    part[2 * blockIdx.x + 1] = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
  }
}

// get_ray_bundle (nerf_utils.py:28-93) at ray r = (image b, pixel y, x): origin o, raw direction d
__device__ __forceinline__ void bundle_ray(const nfi_camera& c, long long r, float o[3], float d[3]) {
  const int HW = c.H * c.W;
  const int b = (int)(r / HW);
  const int p = (int)(r % HW);
  const int y = p / c.W, x = p % c.W;
  const float* M = c.cam + b * 16;
  float ii, jj;
  pixel_coords(c, b, x, y, ii, jj);
  if (c.focal) {
    const float f = c.focal[b];
    ii = fdiv(ii, f);
    jj = fdiv(jj, f);
    const float dc[3] = {ii, -jj, -1.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      d[i] = rowdot3(dc, M + i * 4);
      o[i] = M[i * 4 + 3];
    }
  } else {
    const float oc[3] = {ii, -jj, 0.f};
    const float dc[3] = {0.f, 0.f, -1.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      o[i] = fadd(rowdot3(oc, M + i * 4), M[i * 4 + 3]);
      d[i] = fdiv(rowdot3(dc, M + i * 4), M[15]);
    }
  }
}

// the ray bundle alone (the get_ray_bundle seam): ro, raw rd [B*H*W][3]
__global__ void __launch_bounds__(256) ray_bundle_kernel(nfi_camera c, float* __restrict__ ro, float* __restrict__ rd) {
  const long long n = (long long)c.B * c.H * c.W;
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float o[3], d[3];
  bundle_ray(c, r, o, d);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    ro[r * 3 + i] = o[i];
    rd[r * 3 + i] = d[i];
  }
}

__global__ void __launch_bounds__(256) rays_fwd_kernel(nfi_camera c, float sr, float* __restrict__ ro,
                                                       float* __restrict__ rd, float* __restrict__ nearp,
                                                       float* __restrict__ farp, uint32_t* __restrict__ part,
                                                       uint8_t* __restrict__ hitflag) {
  const int HW = c.H * c.W;
  const long long n = (long long)c.B * HW;
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float nr = INFINITY, fr = -INFINITY;
  bool hit = false;
  if (r < n) {
    float o[3], d[3];
    bundle_ray(c, r, o, d);
    // F.normalize: x / clamp_min(||x||, 1e-12)
    const float nrm = fmaxf(tnorm3(d[0], d[1], d[2]), 1e-12f);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      d[i] = fdiv(d[i], nrm);
      ro[r * 3 + i] = o[i];
      rd[r * 3 + i] = d[i];
    }
    // slab test against [-sr, sr]^3 (nerf_utils.py:235-258)
    hit = slab_test(o, d, sr, nr, fr);
    nearp[r] = nr;
    farp[r] = fr;
    hitflag[r] = hit ? 1 : 0;
  }
  // min near / max far over hits of the whole call (nerf_utils.py:260-261)
  block_hit_range(hit, nr, fr, part);
}

// compute_near_far_planes (nerf_utils.py:227-275) on the caller's rays [n][3] (not normalised
// here: the reference takes the directions as given), then rays_fix_kernel
__global__ void __launch_bounds__(256) near_far_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                                       long long n, float sr, float* __restrict__ nearp,
                                                       float* __restrict__ farp, uint32_t* __restrict__ part,
                                                       uint8_t* __restrict__ hitflag) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float nr = INFINITY, fr = -INFINITY;
  bool hit = false;
  if (r < n) {
    const float o[3] = {ro[r * 3 + 0], ro[r * 3 + 1], ro[r * 3 + 2]};
    const float d[3] = {rd[r * 3 + 0], rd[r * 3 + 1], rd[r * 3 + 2]};
    hit = slab_test(o, d, sr, nr, fr);
    nearp[r] = nr;
    farp[r] = fr;
    hitflag[r] = hit ? 1 : 0;
  }
  block_hit_range(hit, nr, fr, part);
}

__global__ void __launch_bounds__(256) rays_fix_kernel(long long n, float* __restrict__ nearp,
                                                       float* __restrict__ farp,
                                                       const uint32_t* __restrict__ part, int nparts,
                                                       const uint8_t* __restrict__ hitflag) {
  __shared__ uint32_t red[2][4];
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < n;
  const bool miss = live && !hitflag[r];
  uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
  if (__syncthreads_or(miss)) {     // a ray of this block missed the box: the call's min / max
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
      kmin = min(kmin, part[2 * i]);
      kmax = max(kmax, part[2 * i + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
      kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    if ((threadIdx.x & 63) == 0) {
      lds_st(&red[0][threadIdx.x >> 6], kmin);
      lds_st(&red[1][threadIdx.x >> 6], kmax);
    }
    __syncthreads();
    kmin = min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3]));
    kmax = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
  }
  if (!live) return;
  float nr = nearp[r], fr = farp[r];
  if (miss) {
    nr = fdecode(kmin);
    fr = fdecode(kmax);
  }
  nr = fmaxf(nr, 0.1f);   // clamp_(min=0.1)  (nerf_utils.py:264-265)
  fr = fmaxf(fr, 0.1f);
  if (fsub(fr, nr) < 1e-3f) fr = fadd(nr, 1e-3f);   // (nerf_utils.py:268-270)
  nearp[r] = nr;
  farp[r] = fr;
}

// Backward of get_ray_bundle + F.normalize (NORM) or of get_ray_bundle alone (the seam: g_rd is the
// gradient of the raw directions); per-pixel partials of d cam / d focal.
template <bool NORM>
__global__ void __launch_bounds__(256) rays_bwd_kernel(nfi_camera c, const float* __restrict__ g_ro,
                                                       const float* __restrict__ g_rd,
                                                       float* __restrict__ contrib) {
  const int HW = c.H * c.W;
  const long long n = (long long)c.B * HW;
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int b = (int)(r / HW);
  const int p = (int)(r % HW);
  const int y = p / c.W, x = p % c.W;
  const float* M = c.cam + b * 16;
  float ii, jj;
  pixel_coords(c, b, x, y, ii, jj);
  float out[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = 0.f;
  float dc[3], d[3];
  float f = 1.f;
  if (c.focal) {
    f = c.focal[b];
    dc[0] = ii / f;
    dc[1] = -(jj / f);
    dc[2] = -1.f;
  } else {
    dc[0] = 0.f;
    dc[1] = 0.f;
    dc[2] = -1.f;
  }
  float u[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) u[i] = dc[0] * M[i * 4 + 0] + dc[1] * M[i * 4 + 1] + dc[2] * M[i * 4 + 2];
  const float c33 = c.focal ? 1.f : M[15];
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = u[i] / c33;
  // normalize backward: g_raw = (g - y (y.g)) / n
  const float nn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  const float nrm = fmaxf(nn, 1e-12f);
  float yv[3], g[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    yv[i] = d[i] / nrm;
    g[i] = g_rd[r * 3 + i];
  }
  const float yg = yv[0] * g[0] + yv[1] * g[1] + yv[2] * g[2];
  float graw[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) graw[i] = !NORM ? g[i] : ((nn > 1e-12f) ? (g[i] - yv[i] * yg) / nrm : g[i] / nrm);
  const float gro[3] = {g_ro[r * 3 + 0], g_ro[r * 3 + 1], g_ro[r * 3 + 2]};
  if (c.focal) {
    // d = sum_k dc[k] M[i][k]
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int k = 0; k < 3; ++k) out[i * 4 + k] = graw[i] * dc[k];
      out[i * 4 + 3] = gro[i];
    }
    float gdc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) gdc[k] = graw[0] * M[0 * 4 + k] + graw[1] * M[1 * 4 + k] + graw[2] * M[2 * 4 + k];
    // dc0 = ii/f, dc1 = -(jj/f)
    out[13] = gdc[0] * (-(ii / f) / f) + gdc[1] * ((jj / f) / f);
  } else {
    const float oc[3] = {ii, -jj, 0.f};
    float gu[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) gu[i] = graw[i] / c33;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int k = 0; k < 3; ++k) out[i * 4 + k] = gro[i] * oc[k] + gu[i] * dc[k];
      out[i * 4 + 3] = gro[i];
    }
    out[12] = -(graw[0] * u[0] + graw[1] * u[1] + graw[2] * u[2]) / (c33 * c33);
  }
  float4* o4 = reinterpret_cast<float4*>(contrib + r * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) o4[i] = make_float4(out[i * 4], out[i * 4 + 1], out[i * 4 + 2], out[i * 4 + 3]);
}

// ---------------------------------------------------------------------------------------
// Deterministic per-image reduction: out[b,k] = sum_m in[b,m,k]
// ---------------------------------------------------------------------------------------
constexpr int SEG_CHUNKS = 64;

__global__ void __launch_bounds__(256) segsum_pass1(const float* __restrict__ in, int M, int K,
                                                    float* __restrict__ part) {
  __shared__ float red[256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int rows = (M + SEG_CHUNKS - 1) / SEG_CHUNKS;
  const int m0 = ch * rows, m1 = min(M, m0 + rows);
  const int per = 256 / K;             // threads per k
  const int tid = threadIdx.x;
  const int k = tid % K, s = tid / K;
  float acc = 0.f;
  if (s < per) {
    // 8 independent partial sums: 8 loads in flight per thread (the grid is only 64 x B blocks)
    float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* src = in + (long long)b * M * K + k;
    int m = m0 + s;
    for (; m + 7 * per < m1; m += 8 * per) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a8[u] += src[(long long)(m + u * per) * K];
    }
    for (; m < m1; m += per) a8[0] += src[(long long)m * K];
    acc = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < K) {
    float t = 0.f;
    for (int j = 0; j < per; ++j) t += red[j * K + tid];
    part[((long long)b * SEG_CHUNKS + ch) * K + tid] = t;
  }
}

__global__ void __launch_bounds__(64) segsum_pass2(const float* __restrict__ part, int K,
                                                   float* __restrict__ out) {
  const int b = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 64) {
    float t = 0.f;
    for (int j = 0; j < SEG_CHUNKS; ++j) t += part[((long long)b * SEG_CHUNKS + j) * K + k];
    out[b * K + k] = t;
  }
}

// ---------------------------------------------------------------------------------------
// Decoder packing (EqualizedLinear gains, stylegan.py:173-176)
// ---------------------------------------------------------------------------------------
template <int NOUT>
__global__ void decoder_pack_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                    const float* __restrict__ w2, const float* __restrict__ b2, float g1,
                                    float g2, float gb, float* __restrict__ dec) {
  using L = DecL<NOUT>;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L::SIZE) return;
  // (w1 [64,32], w2 [NOUT,64] row-major; scaled as EqualizedLinear does, stylegan.py:173-176)
  auto W1 = [&](int h, int c) { return w1[h * NC + c] * g1; };
  auto W2 = [&](int o, int h) { return (o < NOUT) ? w2[o * NH + h] * g2 : 0.f; };
  float v = 0.f;
  if (t < L::DB1) {
    const int hb = t / 512, l = (t / 8) % 64, k = t % 8;
    v = W1(16 * hb + (l & 15), 8 * (l >> 4) + k);
  } else if (t < L::DT2) {
    const int u = t - L::DB1, hb = u / 256, l = (u / 4) % 64, r = u % 4;
    v = b1[16 * hb + 4 * (l >> 4) + r] * gb;
  } else if (t < L::DT3) {
    const int u = t - L::DT2, ob = u / 1024, hb = (u / 256) % 4, l = (u / 4) % 64, r = u % 4;
    v = W2(16 * ob + (l & 15), 16 * hb + 4 * (l >> 4) + r);
  } else if (t < L::DT4) {
    const int u = t - L::DT3, hb = u / (64 * L::KTP), l = (u / L::KTP) % 64, k = u % L::KTP;
    v = (k < L::KT) ? W2(4 * k + (l >> 4), 16 * hb + (l & 15)) : 0.f;
  } else if (t < L::DB2) {
    const int u = t - L::DT4, cb = u / 1024, hb = (u / 256) % 4, l = (u / 4) % 64, r = u % 4;
    v = W1(16 * hb + 4 * (l >> 4) + r, 16 * cb + (l & 15));
  } else if (t < L::DT1S) {
    const int k = t - L::DB2;
    v = (k < NOUT) ? b2[k] * gb : 0.f;
  } else if (t < L::DB1S) {
    const int u = t - L::DT1S, hb = u / 512, l = (u / 8) % 64, k = u % 8;
    v = W1(16 * hb + (l & 15), 8 * (l >> 4) + k) * 1.44269504f;
  } else {
    const int u = t - L::DB1S, hb = u / 256, l = (u / 4) % 64, r = u % 4;
    v = (b1[16 * hb + 4 * (l >> 4) + r] * gb) * 1.44269504f;
  }
  dec[t] = v;
}

// The inversion decoder's split-f16 tables (DecH, nfi_common.h): one workgroup finds each
// matrix's power-of-two scale, then writes the hi / lo halves of every scaled weight.
__device__ __forceinline__ unsigned short f16_bits(float v) { return __builtin_bit_cast(unsigned short, (_Float16)v); }
// hi (part 0) or lo (part 1) half of v: hi = f16(v), lo = f16(v - hi), round-to-nearest each
__device__ __forceinline__ unsigned short f16_part(float v, int part) {
  const _Float16 h = (_Float16)v;
  return part ? f16_bits(v - (float)h) : __builtin_bit_cast(unsigned short, h);
}
// exponent e with m 2^e in [2^(top-1), 2^top) (0 for m = 0), kept within +-100
__device__ __forceinline__ int pow2_exp(float m, int top) {
  if (!(m > 0.f) || !isfinite(m)) return 0;
  int E;
  frexpf(m, &E);
  return min(max(top - E, -100), 100);
}

__global__ void __launch_bounds__(256) decoder_pack_h_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                             const float* __restrict__ w2, const float* __restrict__ b2,
                                                             float g1, float g2, float gb, float* __restrict__ dec) {
  using H = DecH;
  __shared__ float red[3][256];
  const int t = threadIdx.x;
  auto W1 = [&](int h, int c) { return w1[h * NC + c] * g1; };
  auto W2 = [&](int o, int h) { return (o < NO) ? w2[o * NH + h] * g2 : 0.f; };
  float m1 = 0.f, m2 = 0.f, c3 = 0.f;
  for (int i = t; i < NH * NC; i += 256) m1 = fmaxf(m1, fabsf(W1(i / NC, i % NC)));
  for (int i = t; i < NO * NH; i += 256) m2 = fmaxf(m2, fabsf(W2(i / NH, i % NH)));
  if (t < NH)
    for (int o = 0; o < NO; ++o) c3 += fabsf(W2(o, t));
  lds_st(&red[0][t], m1);
  lds_st(&red[1][t], m2);
  lds_st(&red[2][t], c3);
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
      for (int k = 0; k < 3; ++k) lds_st(&red[k][t], fmaxf(red[k][t], red[k][t + w]));
    __syncthreads();
  }
  m1 = red[0][0];
  m2 = red[1][0];
  c3 = red[2][0];
  const int e1 = pow2_exp(m1, 15), e2 = pow2_exp(m2 * 0.69314718f, 15), e3 = pow2_exp(m2, 7), e4 = e1;
  // hidden unit of K-step kb at k = 8q + j
  auto hk = [](int kb, int q, int j) { return 16 * (2 * kb + (j >> 2)) + 4 * q + (j & 3); };
  // one table dword: the hi (part 0) or lo (part 1) halves of two consecutive operand elements
  auto pair = [](float v0, float v1, int part) {
    return __builtin_bit_cast(float, (unsigned)f16_part(v0, part) | ((unsigned)f16_part(v1, part) << 16));
  };
  for (int i = t; i < H::SIZE; i += 256) {
    float v = 0.f;
    if (i < H::B1S) {
      const int hb = i / 512, l = (i / 8) % 64, w = i % 8, part = w >> 2, j = 2 * (w & 3);
      const int row = 16 * hb + (l & 15), c = 8 * (l >> 4) + j;
      v = pair(ldexpf(W1(row, c), e1), ldexpf(W1(row, c + 1), e1), part);
    } else if (i < H::H2) {
      const int u = i - H::B1S, hb = u / 256, l = (u / 4) % 64, r = u % 4;
      v = (b1[16 * hb + 4 * (l >> 4) + r] * gb) * 1.44269504f;
    } else if (i < H::H3) {
      const int u = i - H::H2, kb = u / 512, l = (u / 8) % 64, w = u % 8, part = w >> 2, j = 2 * (w & 3);
      const int o = l & 15, q = l >> 4;
      // (times ln 2: the forward's hidden activations arrive as softplus / ln 2, nfi_render.hip)
      v = pair(ldexpf(W2(o, hk(kb, q, j)) * 0.69314718f, e2), ldexpf(W2(o, hk(kb, q, j + 1)) * 0.69314718f, e2),
               part);
    } else if (i < H::H4) {
      const int u = i - H::H3, hb = u / 256, l = (u / 4) % 64, w = u % 4;
      const int h = 16 * hb + (l & 15), k = 8 * (l >> 4) + 2 * w, part = k >= 16, o = k & 15;
      v = pair(ldexpf(W2(o, h), e3), ldexpf(W2(o + 1, h), e3), part);
    } else if (i < H::B2) {
      const int u = i - H::H4, cb = u / 1024, kb = (u / 512) % 2, l = (u / 8) % 64, w = u % 8;
      const int part = w >> 2, j = 2 * (w & 3), c = 16 * cb + (l & 15), q = l >> 4;
      v = pair(ldexpf(W1(hk(kb, q, j), c), e4), ldexpf(W1(hk(kb, q, j + 1), c), e4), part);
    } else if (i < H::SC) {
      const int k = i - H::B2;
      v = (k < NO) ? b2[k] * gb : 0.f;
    } else {
      const int k = i - H::SC;
      v = (k == 0) ? ldexpf(1.44269504f, -e1)
        : (k == 1) ? ldexpf(1.f, -e2)
        : (k == 2) ? ldexpf(c3, e3)
        : (k == 3) ? ldexpf(1.f, -(e3 + e4)) : 0.f;
    }
    dec[i] = v;
  }
}

// ---------------------------------------------------------------------------------------
// Plane layout: [B,3,32,R,R] <-> [B,3,R,R,32]  (LDS-tiled transpose, 32 ch x 64 texels)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) planes_c2t_kernel(const float* __restrict__ src, int RR,
                                                         float* __restrict__ dst) {
  __shared__ float tile[NC][65];
  const long long bq = blockIdx.y;              // b*3 + q
  const int t0 = blockIdx.x * 64;
  const float* s = src + bq * NC * (long long)RR;
  float* d = dst + bq * NC * (long long)RR;
  for (int i = threadIdx.x; i < NC * 64; i += 256) {
    const int c = i / 64, t = i % 64;
    tile[c][t] = (t0 + t < RR) ? s[(long long)c * RR + t0 + t] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NC * 64; i += 256) {
    const int t = i / NC, c = i % NC;
    if (t0 + t < RR) d[(long long)(t0 + t) * NC + c] = tile[c][t];
  }
}

__global__ void __launch_bounds__(256) planes_t2c_kernel(const float* __restrict__ src, int RR,
                                                         float* __restrict__ dst) {
  __shared__ float tile[NC][65];
  const long long bq = blockIdx.y;
  const int t0 = blockIdx.x * 64;
  const float* s = src + bq * NC * (long long)RR;
  float* d = dst + bq * NC * (long long)RR;
  for (int i = threadIdx.x; i < NC * 64; i += 256) {
    const int t = i / NC, c = i % NC;
    tile[c][t] = (t0 + t < RR) ? s[(long long)(t0 + t) * NC + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NC * 64; i += 256) {
    const int c = i / 64, t = i % 64;
    if (t0 + t < RR) d[(long long)c * RR + t0 + t] = tile[c][t];
  }
}

// ---------------------------------------------------------------------------------------
// The inversion step's pose algebra (run.py:2262-2266 -> pose_utils.py:48-78) in one launch each way:
// cam2world [b,4,4] and focal [b] from the optimised (z0, t2, s, q), q through F.normalize first;
// and the post-step projections (run.py:2300-2306).  One thread per image (the batch is a handful
// of images: this replaces ~35 scalar-sized ATen kernels per step, forward and backward).
// ---------------------------------------------------------------------------------------
// r = the row-major rotation matrix of the unit quaternion (w, x, y, z); the reference's matrix is
// its transpose (pose_utils.py:41-45 rotates the rows of the identity): R[i][j] = r[3j + i].
__device__ __forceinline__ void quat_r(const float n[4], float r[9]) {
  const float w = n[0], x = n[1], y = n[2], z = n[3];
  r[0] = 1.f - 2.f * (y * y + z * z);
  r[1] = 2.f * (x * y - w * z);
  r[2] = 2.f * (x * z + w * y);
  r[3] = 2.f * (x * y + w * z);
  r[4] = 1.f - 2.f * (x * x + z * z);
  r[5] = 2.f * (y * z - w * x);
  r[6] = 2.f * (x * z - w * y);
  r[7] = 2.f * (y * z + w * x);
  r[8] = 1.f - 2.f * (x * x + y * y);
}

struct PoseIn {
  float n[4];      // F.normalize(q)
  float qnorm;     // max(||q||, 1e-12)
  float t3[3];     // (t2 / s, f / s) or (t2, 1) / s
  float ez;        // exp(z0) (0 without z0)
  float R[3][3];
};

__device__ __forceinline__ PoseIn pose_in(const float* z0, const float* t2, const float* s, const float* q, int b) {
  PoseIn P;
  const float q0 = q[4 * b], q1 = q[4 * b + 1], q2 = q[4 * b + 2], q3 = q[4 * b + 3];
  P.qnorm = fmaxf(sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3), 1e-12f);
  P.n[0] = q0 / P.qnorm;
  P.n[1] = q1 / P.qnorm;
  P.n[2] = q2 / P.qnorm;
  P.n[3] = q3 / P.qnorm;
  float r[9];
  quat_r(P.n, r);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) P.R[i][j] = r[3 * j + i];
  const float sv = s[b];
  P.ez = z0 ? expf(z0[b]) : 0.f;
  const float f = z0 ? 1.f + P.ez : 1.f;
  P.t3[0] = t2[2 * b] / sv;
  P.t3[1] = t2[2 * b + 1] / sv;
  P.t3[2] = f / sv;
  return P;
}

__global__ void pose_fwd_kernel(const float* __restrict__ z0, const float* __restrict__ t2,
                                const float* __restrict__ s, const float* __restrict__ q, int B, int flipped,
                                float* __restrict__ cam, float* __restrict__ focal) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const PoseIn P = pose_in(z0, t2, s, q, b);
  float* m = cam + 16 * b;
  const float sg = flipped ? -1.f : 1.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float c3 = P.R[i][0] * P.t3[0] + P.R[i][1] * P.t3[1] + P.R[i][2] * P.t3[2];
    m[4 * i + 0] = P.R[i][0];
    m[4 * i + 1] = sg * P.R[i][1];
    m[4 * i + 2] = sg * P.R[i][2];
    m[4 * i + 3] = sg * c3;
  }
  m[12] = 0.f;
  m[13] = 0.f;
  m[14] = 0.f;
  m[15] = 1.f;
  if (z0 && focal) focal[b] = (1.f + P.ez) / 2.f;
}

// d cam2world [b,4,4] (+ d focal [b]) -> d z0, d t2, d s, d q (each written, not accumulated)
__global__ void pose_bwd_kernel(const float* __restrict__ z0, const float* __restrict__ t2,
                                const float* __restrict__ s, const float* __restrict__ q, int B, int flipped,
                                const float* __restrict__ g_cam, const float* __restrict__ g_focal,
                                float* __restrict__ d_z0, float* __restrict__ d_t2, float* __restrict__ d_s,
                                float* __restrict__ d_q) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const PoseIn P = pose_in(z0, t2, s, q, b);
  float G[3][4];
  const float sg = flipped ? -1.f : 1.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) G[i][j] = (j == 0 ? 1.f : sg) * g_cam[16 * b + 4 * i + j];
  // mat[i][3] = sum_j R[i][j] t3[j]
  float dr[9], dt3[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      dr[3 * j + i] = G[i][j] + G[i][3] * P.t3[j];
      dt3[j] += G[i][3] * P.R[i][j];
    }
  const float sv = s[b];
  d_t2[2 * b] = dt3[0] / sv;
  d_t2[2 * b + 1] = dt3[1] / sv;
  d_s[b] = -(dt3[0] * P.t3[0] + dt3[1] * P.t3[1] + dt3[2] * P.t3[2]) / sv;
  if (z0 && d_z0) {
    const float df = dt3[2] / sv + (g_focal ? 0.5f * g_focal[b] : 0.f);
    d_z0[b] = df * P.ez;
  }
  // r(n): d r / d n of the quadratic forms in quat_r
  const float w = P.n[0], x = P.n[1], y = P.n[2], z = P.n[3];
  const float dw = 2.f * (-z * dr[1] + y * dr[2] + z * dr[3] - y * dr[6] - x * dr[5] + x * dr[7]);
  const float dx = 2.f * (y * dr[1] + z * dr[2] + y * dr[3] - 2.f * x * dr[4] - w * dr[5] + z * dr[6] +
                          w * dr[7] - 2.f * x * dr[8]);
  const float dy = 2.f * (-2.f * y * dr[0] + x * dr[1] + w * dr[2] + x * dr[3] + z * dr[5] - w * dr[6] +
                          z * dr[7] - 2.f * y * dr[8]);
  const float dz = 2.f * (-2.f * z * dr[0] - w * dr[1] + x * dr[2] + w * dr[3] - 2.f * z * dr[4] + y * dr[5] +
                          x * dr[6] + y * dr[7]);
  // F.normalize backward: (g - n (n . g)) / max(||q||, eps) (the clamp passes no gradient below eps)
  const float dn = w * dw + x * dx + y * dy + z * dz;
  const bool above = P.qnorm > 1e-12f;
  d_q[4 * b + 0] = (dw - (above ? w * dn : 0.f)) / P.qnorm;
  d_q[4 * b + 1] = (dx - (above ? x * dn : 0.f)) / P.qnorm;
  d_q[4 * b + 2] = (dy - (above ? y * dn : 0.f)) / P.qnorm;
  d_q[4 * b + 3] = (dz - (above ? z * dn : 0.f)) / P.qnorm;
}

// after the optimiser step (run.py:2300-2306): q <- F.normalize(q), z0 <- clamp(z0, -4, 4), s <- |s|
__global__ void pose_project_kernel(float* __restrict__ z0, float* __restrict__ s, float* __restrict__ q, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float q0 = q[4 * b], q1 = q[4 * b + 1], q2 = q[4 * b + 2], q3 = q[4 * b + 3];
  const float n = fmaxf(sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3), 1e-12f);
  q[4 * b] = q0 / n;
  q[4 * b + 1] = q1 / n;
  q[4 * b + 2] = q2 / n;
  q[4 * b + 3] = q3 / n;
  if (z0) z0[b] = fminf(fmaxf(z0[b], -4.f), 4.f);
  if (s) s[b] = fabsf(s[b]);
}

}  // namespace nfi

using namespace nfi;

extern "C" {

static_assert(DecH::SIZE == NFI_DEC_SIZE && DecL<NOV>::SIZE == NFI_DEC_SIZE_VIEWDIR, "nfi.h decoder sizes");
int32_t nfi_abi_version(void) { return NFI_ABI_VERSION; }
const char* nfi_last_error(void) { return nfi::g_err.c_str(); }

static int check_cam(const nfi_camera* c) {
  NFI_REQUIRE(c && c->cam, "camera: null cam pointer");
  NFI_REQUIRE(c->B > 0 && c->H > 0 && c->W > 0, "camera: bad shape B=%d H=%d W=%d", c->B, c->H, c->W);
  return NFI_OK;
}

int32_t nfi_rays_forward(const nfi_camera* cam, float scene_range, float* ro, float* rd, float* near_,
                         float* far_, uint32_t* ws, void* stream) {
  int e = check_cam(cam);
  if (e) return e;
  NFI_REQUIRE(ro && rd && near_ && far_ && ws, "rays_forward: null output");
  NFI_REQUIRE(scene_range > 0.f && std::isfinite(scene_range), "rays_forward: bad scene_range");
  hipStream_t s = (hipStream_t)stream;
  const long long n = (long long)cam->B * cam->H * cam->W;
  // ws layout (within the documented 2 + B*H*W words): [0, 2 blocks) = per-block (min, max) keys,
  // then one hit byte per ray
  const int blocks = (int)((n + 255) / 256);
  uint32_t* part = ws;
  uint8_t* hit = reinterpret_cast<uint8_t*>(ws + 2 * (long long)blocks);
  rays_fwd_kernel<<<blocks, 256, 0, s>>>(*cam, scene_range, ro, rd, near_, far_, part, hit);
  NFI_CHECK_LAUNCH("rays_fwd_kernel");
  rays_fix_kernel<<<blocks, 256, 0, s>>>(n, near_, far_, part, blocks, hit);
  NFI_CHECK_LAUNCH("rays_fix_kernel");
  return NFI_OK;
}

int64_t nfi_near_far_workspace_bytes(int64_t n) { return n <= 0 ? -1 : 8 * ((n + 255) / 256) + n; }

int32_t nfi_near_far(const float* ro, const float* rd, int64_t n, float scene_range, float* near_, float* far_,
                     void* ws, void* stream) {
  NFI_REQUIRE(ro && rd && near_ && far_ && ws, "near_far: null pointer");
  NFI_REQUIRE(n > 0, "near_far: no rays (n=%lld): the reference's min() of an empty tensor raises",
              (long long)n);
  NFI_REQUIRE(scene_range > 0.f && std::isfinite(scene_range), "near_far: bad scene_range");
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (int)((n + 255) / 256);
  uint32_t* part = reinterpret_cast<uint32_t*>(ws);
  uint8_t* hit = reinterpret_cast<uint8_t*>(part + 2 * (long long)blocks);
  near_far_kernel<<<blocks, 256, 0, s>>>(ro, rd, n, scene_range, near_, far_, part, hit);
  NFI_CHECK_LAUNCH("near_far_kernel");
  rays_fix_kernel<<<blocks, 256, 0, s>>>(n, near_, far_, part, blocks, hit);
  NFI_CHECK_LAUNCH("rays_fix_kernel");
  return NFI_OK;
}

int32_t nfi_rays_backward(const nfi_camera* cam, const float* g_ro, const float* g_rd, float* contrib,
                          void* stream) {
  int e = check_cam(cam);
  if (e) return e;
  NFI_REQUIRE(g_ro && g_rd && contrib, "rays_backward: null pointer");
  const long long n = (long long)cam->B * cam->H * cam->W;
  rays_bwd_kernel<true><<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(*cam, g_ro, g_rd, contrib);
  NFI_CHECK_LAUNCH("rays_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_ray_bundle(const nfi_camera* cam, float* ro, float* rd, void* stream) {
  int e = check_cam(cam);
  if (e) return e;
  NFI_REQUIRE(ro && rd, "ray_bundle: null output");
  const long long n = (long long)cam->B * cam->H * cam->W;
  ray_bundle_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(*cam, ro, rd);
  NFI_CHECK_LAUNCH("ray_bundle_kernel");
  return NFI_OK;
}

int32_t nfi_ray_bundle_backward(const nfi_camera* cam, const float* g_ro, const float* g_rd, float* contrib,
                                void* stream) {
  int e = check_cam(cam);
  if (e) return e;
  NFI_REQUIRE(g_ro && g_rd && contrib, "ray_bundle_backward: null pointer");
  const long long n = (long long)cam->B * cam->H * cam->W;
  rays_bwd_kernel<false><<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(*cam, g_ro, g_rd, contrib);
  NFI_CHECK_LAUNCH("rays_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_segment_sum(const float* in, int32_t B, int32_t M, int32_t K, float* out, float* ws,
                        void* stream) {
  NFI_REQUIRE(in && out && ws, "segment_sum: null pointer");
  NFI_REQUIRE(B > 0 && M > 0 && K > 0 && K <= 256, "segment_sum: bad shape B=%d M=%d K=%d", B, M, K);
  hipStream_t s = (hipStream_t)stream;
  segsum_pass1<<<dim3(SEG_CHUNKS, B), 256, 0, s>>>(in, M, K, ws);
  NFI_CHECK_LAUNCH("segsum_pass1");
  segsum_pass2<<<B, 64, 0, s>>>(ws, K, out);
  NFI_CHECK_LAUNCH("segsum_pass2");
  return NFI_OK;
}

int32_t nfi_decoder_pack(const float* w1, const float* b1, const float* w2, const float* b2, float g1,
                         float g2, float gb, float* dec, void* stream) {
  return nfi_decoder_pack_n(w1, b1, w2, b2, NO, g1, g2, gb, dec, stream);
}

int64_t nfi_decoder_size(int32_t nout) {
  if (nout == NO) return DecH::SIZE;
  if (nout == NOV) return DecL<NOV>::SIZE;
  return -1;
}

int32_t nfi_decoder_pack_n(const float* w1, const float* b1, const float* w2, const float* b2, int32_t nout,
                           float g1, float g2, float gb, float* dec, void* stream) {
  NFI_REQUIRE(w1 && b1 && w2 && b2 && dec, "decoder_pack: null pointer");
  NFI_REQUIRE(nout == NO || nout == NOV, "decoder_pack: nout must be %d or %d (got %d)", NO, NOV, nout);
  if (nout == NO)
    decoder_pack_h_kernel<<<1, 256, 0, (hipStream_t)stream>>>(w1, b1, w2, b2, g1, g2, gb, dec);
  else
    decoder_pack_kernel<NOV><<<(DecL<NOV>::SIZE + 255) / 256, 256, 0, (hipStream_t)stream>>>(w1, b1, w2, b2, g1,
                                                                                              g2, gb, dec);
  NFI_CHECK_LAUNCH("decoder_pack_kernel");
  return NFI_OK;
}

int32_t nfi_planes_to_texel_major(const float* src, int32_t B, int32_t R, float* dst, void* stream) {
  NFI_REQUIRE(src && dst && B > 0 && R > 1, "planes_to_texel_major: bad args");
  const int RR = R * R;
  planes_c2t_kernel<<<dim3((RR + 63) / 64, B * 3), 256, 0, (hipStream_t)stream>>>(src, RR, dst);
  NFI_CHECK_LAUNCH("planes_c2t_kernel");
  return NFI_OK;
}

int32_t nfi_planes_to_channel_major(const float* src, int32_t B, int32_t R, float* dst, void* stream) {
  NFI_REQUIRE(src && dst && B > 0 && R > 1, "planes_to_channel_major: bad args");
  const int RR = R * R;
  planes_t2c_kernel<<<dim3((RR + 63) / 64, B * 3), 256, 0, (hipStream_t)stream>>>(src, RR, dst);
  NFI_CHECK_LAUNCH("planes_t2c_kernel");
  return NFI_OK;
}

int32_t nfi_pose_forward(const float* z0, const float* t2, const float* s, const float* q, int32_t B,
                         int32_t camera_flipped, float* cam2world, float* focal, void* stream) {
  NFI_REQUIRE(t2 && s && q && cam2world && B > 0, "pose_forward: bad args (B=%d)", B);
  NFI_REQUIRE(!z0 || focal, "pose_forward: z0 given without a focal output");
  pose_fwd_kernel<<<(B + 63) / 64, 64, 0, (hipStream_t)stream>>>(z0, t2, s, q, B, camera_flipped != 0, cam2world,
                                                                 focal);
  NFI_CHECK_LAUNCH("pose_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_pose_backward(const float* z0, const float* t2, const float* s, const float* q, int32_t B,
                          int32_t camera_flipped, const float* g_cam2world, const float* g_focal, float* d_z0,
                          float* d_t2, float* d_s, float* d_q, void* stream) {
  NFI_REQUIRE(t2 && s && q && g_cam2world && d_t2 && d_s && d_q && B > 0, "pose_backward: bad args (B=%d)", B);
  NFI_REQUIRE(!z0 || d_z0, "pose_backward: z0 given without a d_z0 output");
  pose_bwd_kernel<<<(B + 63) / 64, 64, 0, (hipStream_t)stream>>>(z0, t2, s, q, B, camera_flipped != 0,
                                                                 g_cam2world, g_focal, d_z0, d_t2, d_s, d_q);
  NFI_CHECK_LAUNCH("pose_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_pose_project(float* z0, float* s, float* q, int32_t B, void* stream) {
  NFI_REQUIRE(q && B > 0, "pose_project: bad args (B=%d)", B);
  pose_project_kernel<<<(B + 63) / 64, 64, 0, (hipStream_t)stream>>>(z0, s, q, B);
  NFI_CHECK_LAUNCH("pose_project_kernel");
  return NFI_OK;
}

}  // extern "C"
