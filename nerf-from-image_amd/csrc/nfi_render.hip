// Fused volume renderer of the SDF-NeRF inversion loop (reference: run.py:176-350,
// lib/nerf_utils.py, models/generator.py:288-331,587-681), forward and backward, for
// MI355X (gfx950, CDNA4, wave64).
//
// Work decomposition: one wave64 per ray, four rays per 256-thread workgroup.  Per-ray state
// (sample depths, densities, colours, CDF, merged order) lives in lanes and in the wave's
// private LDS slice; the only HBM traffic per sample is the tri-plane tap (fwd), its
// re-gather + scatter-add (bwd), and a few bytes of per-ray I/O.
//
// Tri-plane taps are gathered "channel-on-lane": for one point, one wave instruction reads
// one bilinear row pair = 2 texels x 32 channels = 256 contiguous bytes (texel-major planes),
// lanes 0-31 = texel x0, lanes 32-63 = texel x0+1.  The interpolated 32-d feature is
// transposed through LDS so that the 32->64->11 decoder runs point-on-lane with its weights
// in SGPRs (wave-uniform scalar loads).  Backward scatters d planes with the same 256-byte
// wave-instruction shape, which is the full-rate shape of gfx950 float atomics.
#include <cmath>

#include "nfi_common.h"
#include "nfi_host.h"

namespace nfi {

constexpr int XS = 36;                  // LDS row stride (floats) of the point x channel tile
constexpr int XTILE = WAVE * XS;        // 2304 floats

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// v + v(lane ^ 32), in every lane (gfx950 v_permlane32_swap).
__device__ __forceinline__ float sum_halves(float v) {
  auto s = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(s[0]) + __int_as_float(s[1]);
}

// ---------------------------------------------------------------------------------------
// Per-point bilinear parameters of one plane: F.grid_sample(bilinear, border,
// align_corners=True) as ATen's CPU kernel computes them (unnormalize (g+1)*(R-1)/2, clip to
// [0,R-1], floor, w = x - x0, e = 1 - w; grid-grad multiplier (R-1)/2 strictly inside).
// ---------------------------------------------------------------------------------------
struct PlaneP {
  int tex;          // y0*R + x0 | (x0 < R-1) << 20 | (y0 < R-1) << 21
  float e, w, s, n;
  float gxm, gym;
};

__device__ __forceinline__ void plane_params(float gu, float gv, int R, PlaneP& p) {
  const float Rm1 = (float)(R - 1);
  const float half = Rm1 / 2.f;
  float ix = (gu + 1.f) * half;
  float iy = (gv + 1.f) * half;
  p.gxm = (ix > 0.f && ix < Rm1) ? half : 0.f;
  p.gym = (iy > 0.f && iy < Rm1) ? half : 0.f;
  ix = fminf(Rm1, fmaxf(ix, 0.f));
  iy = fminf(Rm1, fmaxf(iy, 0.f));
  const float x0 = floorf(ix), y0 = floorf(iy);
  p.w = ix - x0;
  p.e = 1.f - p.w;
  p.n = iy - y0;
  p.s = 1.f - p.n;
  const int xi = (int)x0, yi = (int)y0;
  p.tex = (yi * R + xi) | ((xi < R - 1) ? (1 << 20) : 0) | ((yi < R - 1) ? (1 << 21) : 0);
}

struct PointP {
  float cx[3];      // normalized coords p / scene_range
  float mask;       // 1 outside [-1,1]^3 (generator.py:605-607)
  PlaneP pl[3];     // xy, xz, yz (generator.py:312-326)
};

__device__ __forceinline__ void point_params(const float o[3], const float d[3], float t, float sr, int R,
                                             PointP& P) {
#pragma unroll
  for (int k = 0; k < 3; ++k) P.cx[k] = (o[k] + d[k] * t) / sr;
  P.mask = (fabsf(P.cx[0]) > 1.f || fabsf(P.cx[1]) > 1.f || fabsf(P.cx[2]) > 1.f) ? 1.f : 0.f;
  plane_params(P.cx[0], P.cx[1], R, P.pl[0]);
  plane_params(P.cx[0], P.cx[2], R, P.pl[1]);
  plane_params(P.cx[1], P.cx[2], R, P.pl[2]);
}

struct PlaneView {
  const float* __restrict__ base;   // planes of this image
  int sq, st, R;
};

// Gather + interpolate + mean-of-3 for points 0..npts-1 of the wave (point j's parameters live
// in lane j); writes X[j][c] (j < npts) into the wave's LDS tile.
__device__ __forceinline__ void gather_features(const PlaneView& pv, const PointP& P, int npts,
                                                float* __restrict__ X) {
  const int l = lane_id();
  const int dx = l >> 5, c = l & 31;
#pragma unroll 2
  for (int j = 0; j < npts; ++j) {
    float E[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int pk = readlane(P.pl[q].tex, j);
      const float e = readlane(P.pl[q].e, j), w = readlane(P.pl[q].w, j);
      const float s = readlane(P.pl[q].s, j), n = readlane(P.pl[q].n, j);
      const int t0 = (pk & 0xFFFFF) + (dx ? ((pk >> 20) & 1) : 0);
      const int t1 = t0 + (((pk >> 21) & 1) ? pv.R : 0);
      const float* b = pv.base + q * pv.sq + c;
      const float v0 = b[t0 * pv.st];
      const float v1 = b[t1 * pv.st];
      const float wx = dx ? w : e;
      E[q] = sum_halves(v0 * (s * wx) + v1 * (n * wx));
    }
    if (l < 32) X[j * XS + c] = ((E[0] + E[1]) + E[2]) / 3.f;
  }
}

__device__ __forceinline__ void load_row(const float* __restrict__ X, int row, float x[NC]) {
  const float4* r = reinterpret_cast<const float4*>(X + row * XS);
#pragma unroll
  for (int k = 0; k < NC / 4; ++k) {
    const float4 v = r[k];
    x[4 * k + 0] = v.x;
    x[4 * k + 1] = v.y;
    x[4 * k + 2] = v.z;
    x[4 * k + 3] = v.w;
  }
}

__device__ __forceinline__ void store_row(float* __restrict__ X, int row, const float x[NC]) {
  float4* r = reinterpret_cast<float4*>(X + row * XS);
#pragma unroll
  for (int k = 0; k < NC / 4; ++k) r[k] = make_float4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
}

// Softplus(beta=1, threshold=20) (generator.py:297) and its derivative (ATen softplus_backward).
__device__ __forceinline__ float softplus(float z) {
  const float u = __expf(z);
  const float up = 1.f + u;
  const float dd = up - 1.f;
  const float l1p = (dd == 0.f) ? u : __logf(up) * (u / dd);   // accurate log1p(u)
  return (z > 20.f) ? z : l1p;
}
__device__ __forceinline__ float softplus_grad(float z) {
  const float u = __expf(z);
  return (z > 20.f) ? 1.f : u / (u + 1.f);
}

__device__ __forceinline__ float dot32(const float x[NC], const float* __restrict__ w) {
  float z0 = 0.f, z1 = 0.f, z2 = 0.f, z3 = 0.f;
#pragma unroll
  for (int c = 0; c < NC; c += 4) {
    z0 = fmaf(x[c + 0], w[c + 0], z0);
    z1 = fmaf(x[c + 1], w[c + 1], z1);
    z2 = fmaf(x[c + 2], w[c + 2], z2);
    z3 = fmaf(x[c + 3], w[c + 3], z3);
  }
  return (z0 + z1) + (z2 + z3);
}

// TriplanarDecoder.net (generator.py:295-299): y = W2s softplus(W1s x + b1) + b2.
__device__ __forceinline__ void mlp_forward(const float* __restrict__ dec, const float x[NC], float y[NO]) {
  float acc[NO];
#pragma unroll
  for (int k = 0; k < NO; ++k) acc[k] = 0.f;
#pragma unroll 2
  for (int o = 0; o < NH; ++o) {
    const float* u = dec + o * DEC_UNIT;
    const float h = softplus(dot32(x, u) + u[DEC_B1]);
#pragma unroll
    for (int k = 0; k < NO; ++k) acc[k] = fmaf(h, u[DEC_W2T + k], acc[k]);
  }
#pragma unroll
  for (int k = 0; k < NO; ++k) y[k] = acc[k] + dec[DEC_B2 + k];
}

// Input-gradient of the decoder (its weights are frozen during inversion, run.py:630-632).
__device__ __forceinline__ void mlp_backward(const float* __restrict__ dec, const float x[NC],
                                             const float gy[NO], float gx[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) gx[c] = 0.f;
#pragma unroll 2
  for (int o = 0; o < NH; ++o) {
    const float* u = dec + o * DEC_UNIT;
    const float z = dot32(x, u) + u[DEC_B1];
    float gh = 0.f;
#pragma unroll
    for (int k = 0; k < NO; ++k) gh = fmaf(gy[k], u[DEC_W2T + k], gh);
    const float gz = gh * softplus_grad(z);
#pragma unroll
    for (int c = 0; c < NC; ++c) gx[c] = fmaf(gz, u[c], gx[c]);
  }
}

// Head: sigma = (1/alpha) * laplace_cdf(-d, beta) * (1 - mask)  (generator.py:629-636, 30-33)
//       rgb   = softmax(features) @ palette                    (generator.py:668-679)
struct Head {
  float sigma;
  float rgb[3];
  float p[NA];
};

__device__ __forceinline__ void head_forward(const float y[NO], float mask, float inv_alpha, float beta,
                                             const float* __restrict__ pal, Head& h) {
  const float xn = -y[0];
  const float ex = expf(-fabsf(xn) / beta);
  const float cdf = 0.5f + 0.5f * tsign(xn) * (1.f - ex);
  h.sigma = inv_alpha * (cdf * (1.f - mask));
  float m = y[1];
#pragma unroll
  for (int k = 2; k <= NA; ++k) m = fmaxf(m, y[k]);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    h.p[k] = __expf(y[1 + k] - m);
    sum += h.p[k];
  }
#pragma unroll
  for (int k = 0; k < NA; ++k) h.p[k] = h.p[k] / sum;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) a = fmaf(h.p[k], pal[k * 3 + c], a);
    h.rgb[c] = a;
  }
}

// ---------------------------------------------------------------------------------------
// Chunked wave scans over per-ray arrays held as v[e] = element (e*64 + lane).
// ---------------------------------------------------------------------------------------
template <int E>
__device__ __forceinline__ void excl_prod(const float (&a)[E], float (&T)[E]) {
  float carry = 1.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float inc = wave_incl_prod(a[e]);
    float ex = __shfl_up(inc, 1);
    if (lane_id() == 0) ex = 1.f;
    T[e] = carry * ex;
    carry = carry * readlane(inc, 63);
  }
}

// ---------------------------------------------------------------------------------------
// Forward kernel
// ---------------------------------------------------------------------------------------
struct RayCtx {
  long long r;
  int b;
  float o[3], d[3];
  float rdn;
  float near_, far_;
};

__device__ __forceinline__ void load_ray(const nfi_render_args& a, long long r, RayCtx& R) {
  R.r = r;
  R.b = (int)(r / a.HW);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    R.o[k] = a.ro[r * 3 + k];
    R.d[k] = a.rd[r * 3 + k];
  }
  R.rdn = sqrtf(R.d[0] * R.d[0] + R.d[1] * R.d[1] + R.d[2] * R.d[2]);   // ray_directions.norm
  R.near_ = a.near_[r];
  R.far_ = a.far_[r];
}

// Evaluate the field at the (up to 64) points t (one per lane; lanes >= npts ignored).
__device__ __forceinline__ void field_eval(const nfi_render_args& a, const PlaneView& pv, const RayCtx& R,
                                           float t, int npts, float* __restrict__ X, float& sigma,
                                           float rgb[3]) {
  PointP P;
  point_params(R.o, R.d, t, a.field.scene_range, pv.R, P);
  gather_features(pv, P, npts, X);
  wave_lds_sync();
  float x[NC];
  load_row(X, lane_id(), x);
  float y[NO];
  mlp_forward(a.field.dec, x, y);
  Head h;
  head_forward(y, P.mask, a.field.inv_alpha, a.field.beta, a.field.palette + R.b * (NA * 3), h);
  sigma = h.sigma;
  rgb[0] = h.rgb[0];
  rgb[1] = h.rgb[1];
  rgb[2] = h.rgb[2];
  wave_lds_sync();
}

template <int S, bool FINE>
struct Cfg {
  static constexpr int SPL = (S + 63) / 64;            // coarse elements per lane
  static constexpr int N = FINE ? 2 * S : S;            // merged samples per ray
  static constexpr int NPL = (N + 63) / 64;
  static constexpr int WAVE_LDS = XTILE + 5 * N + 2 * S + 8;
};

template <int S, bool FINE>
__global__ void __launch_bounds__(256) render_fwd_kernel(nfi_render_args a) {
  using C = Cfg<S, FINE>;
  constexpr int SPL = C::SPL, N = C::N, NPL = C::NPL;
  __shared__ __attribute__((aligned(16))) float lds[4 * C::WAVE_LDS];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= nrays) return;
  float* X = lds + wv * C::WAVE_LDS;
  float* Mt = X + XTILE;          // merged t     [N]
  float* Ms = Mt + N;             // merged sigma [N]
  float* Mc = Ms + N;             // merged rgb   [3][N]
  float* T2 = Mc + 3 * N;         // coarse t [S] then fine t [S] (rank computation) / cdf, bins

  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};

  // ---- stratified coarse depths (nerf_utils.py:104-120) ----
  float tc[SPL], sc[SPL], cc[SPL][3];
#pragma unroll
  for (int e = 0; e < SPL; ++e) {
    const int i = e * 64 + l;
    float t = R.near_;
    if (i < S) {
      t = tlerp(R.near_, R.far_, (float)i / (float)S);
      if (a.randomize) {
        const float u = a.u_coarse ? a.u_coarse[r * S + i] : rng_uniform(a.seed, a.offset, r, i, 0);
        t = t + u * ((R.far_ - R.near_) / (float)S);
      }
      if (a.z_coarse) a.z_coarse[r * S + i] = t;
    }
    tc[e] = t;
    field_eval(a, pv, R, t, min(64, S - e * 64), X, sc[e], cc[e]);
  }

  if constexpr (FINE) {
    // ---- coarse weights, no grad (nerf_utils.py:166-182) ----
    float al[SPL], aa[SPL], T[SPL], w[SPL];
#pragma unroll
    for (int e = 0; e < SPL; ++e) T2[e * 64 + l] = tc[e];
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      float dist = 0.f;
      if (i < S - 1) dist = T2[i + 1] - tc[e];
      dist = dist * R.rdn;
      const float ex = expf(-sc[e] * dist);
      al[e] = 1.f - ex;
      aa[e] = (i < S) ? (1.f - al[e]) + 1e-10f : 1.f;
    }
    excl_prod<SPL>(aa, T);
#pragma unroll
    for (int e = 0; e < SPL; ++e) w[e] = al[e] * T[e];
    wave_lds_sync();
    // ---- EG3D smoothing (run.py:266-272): max_pool1d(2,1,pad 1) -> avg_pool1d(2,1) -> +0.01
    float* Wl = Mt;   // scratch [S]
#pragma unroll
    for (int e = 0; e < SPL; ++e) Wl[e * 64 + l] = w[e];
    wave_lds_sync();
    float sm[SPL];
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      const float wi = w[e];
      const float wp = (i > 0 && i < S) ? Wl[i - 1] : -INFINITY;
      const float wn = (i < S - 1) ? Wl[i + 1] : -INFINITY;
      const float m0 = fmaxf(wp, wi), m1 = fmaxf(wi, wn);
      sm[e] = (m0 + m1) / 2.f + 0.01f;
    }
    wave_lds_sync();
    // ---- sample_pdf (nerf_utils.py:185-224): bins = midpoints [S-1], weights = sm[1..S-2]
    float* cdf = T2 + 0;        // [S-1]
    float* bins = T2 + S;       // [S-1]
#pragma unroll
    for (int e = 0; e < SPL; ++e) Wl[e * 64 + l] = sm[e];
    wave_lds_sync();
    float pw[SPL];
    float tot = 0.f;
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      pw[e] = (i < S - 2) ? Wl[i + 1] + 1e-5f : 0.f;
      tot += pw[e];
    }
    tot = wave_sum(tot);
    // bins from coarse t (still in T2[0..S)); read before overwriting T2
    float mid[SPL];
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      mid[e] = (i < S - 1) ? .5f * (T2[i + 1] + T2[i]) : 0.f;
    }
    wave_lds_sync();
    float carry = 0.f;
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      const float pdf = pw[e] / tot;
      const float inc = wave_incl_sum(pdf) + carry;
      if (i < S - 2) cdf[i + 1] = inc;
      if (i < S - 1) bins[i] = mid[e];
      carry = readlane(inc, 63);
    }
    if (l == 0) cdf[0] = 0.f;
    wave_lds_sync();
    float tf[SPL];
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      float u;
      if (!a.randomize) u = tlinspace01(i, S);
      else u = a.u_fine ? a.u_fine[r * S + min(i, S - 1)] : rng_uniform(a.seed, a.offset, r, i, 1);
      // searchsorted(cdf, u, right=True): number of cdf entries <= u
      int lo = 0, hi = S - 1;
      while (lo < hi) {
        const int mid_ = (lo + hi) >> 1;
        if (cdf[mid_] <= u) lo = mid_ + 1;
        else hi = mid_;
      }
      const int below = max(0, lo - 1), above = min(S - 2, lo);
      const float c0 = cdf[below], c1 = cdf[above];
      const float b0 = bins[below], b1 = bins[above];
      float denom = c1 - c0;
      denom = (denom < 1e-5f) ? 1.f : denom;
      const float tt = (u - c0) / denom;
      tf[e] = b0 + tt * (b1 - b0);
      if (i < S && a.z_fine) a.z_fine[r * S + i] = tf[e];
    }
    wave_lds_sync();
    // ---- fine field evaluation (run.py:283-291) ----
    float sf[SPL], cf[SPL][3];
#pragma unroll
    for (int e = 0; e < SPL; ++e) field_eval(a, pv, R, tf[e], min(64, S - e * 64), X, sf[e], cf[e]);
    // ---- merge: stable sort of cat(z_coarse, z_fine) (run.py:283-288, 312-319) ----
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      if (i < S) {
        T2[i] = tc[e];
        T2[S + i] = tf[e];
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      if (i < S) {
        int rc = 0, rf = 0;
        const float vc = tc[e], vf = tf[e];
        for (int j = 0; j < 2 * S; ++j) {
          const float v = T2[j];
          rc += (v < vc || (v == vc && j < i)) ? 1 : 0;
          rf += (v < vf || (v == vf && j < S + i)) ? 1 : 0;
        }
        Mt[rc] = vc;
        Ms[rc] = sc[e];
        Mt[rf] = vf;
        Ms[rf] = sf[e];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          Mc[k * N + rc] = cc[e][k];
          Mc[k * N + rf] = cf[e][k];
        }
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      if (i < S) {
        Mt[i] = tc[e];
        Ms[i] = sc[e];
#pragma unroll
        for (int k = 0; k < 3; ++k) Mc[k * N + i] = cc[e][k];
      }
    }
  }
  wave_lds_sync();

  // ---- compositing (nerf_utils.py:125-163) ----
  float t[NPL], sg[NPL], al[NPL], aa[NPL], T[NPL];
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    const bool v = i < N;
    t[e] = v ? Mt[i] : 0.f;
    sg[e] = v ? Ms[i] : 0.f;
    const float dist = (i < N - 1) ? (Mt[i + 1] - t[e]) * R.rdn : 0.f;
    const float ex = expf(-sg[e] * dist);
    al[e] = v ? 1.f - ex : 0.f;
    aa[e] = v ? (1.f - al[e]) + 1e-10f : 1.f;
  }
  excl_prod<NPL>(aa, T);
  float sr = 0.f, sgc = 0.f, sb = 0.f, sm = 0.f, sd = 0.f;
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    if (i < N) {
      const float w = al[e] * T[e];
      sr += w * Mc[0 * N + i];
      sgc += w * Mc[1 * N + i];
      sb += w * Mc[2 * N + i];
      sm += w;
      sd += w * t[e];
      a.t_saved[r * N + i] = t[e];
      a.sigma_saved[r * N + i] = sg[e];
#pragma unroll
      for (int k = 0; k < 3; ++k) a.rgb_saved[(r * 3 + k) * N + i] = Mc[k * N + i];
    }
  }
  sr = wave_sum(sr);
  sgc = wave_sum(sgc);
  sb = wave_sum(sb);
  sm = wave_sum(sm);
  sd = wave_sum(sd);
  if (l == 0) {
    const float bg = a.white_bg ? (1.f - sm) : 0.f;
    a.rgb[r * 3 + 0] = sr + bg;
    a.rgb[r * 3 + 1] = sgc + bg;
    a.rgb[r * 3 + 2] = sb + bg;
    a.mask[r] = sm;
    a.depth[r] = sd;
  }
}

// ---------------------------------------------------------------------------------------
// Backward kernel: compositing backward from saved state, then per-sample field backward
// (recompute taps + decoder), scatter-add of d planes, coordinate gradients -> d ro, d rd.
// ---------------------------------------------------------------------------------------
template <int S, bool FINE>
__global__ void __launch_bounds__(256) render_bwd_kernel(nfi_render_args a, nfi_render_grad_args g) {
  using C = Cfg<S, FINE>;
  constexpr int N = C::N, NPL = C::NPL;
  constexpr int WL = XTILE + N + 8;
  __shared__ __attribute__((aligned(16))) float lds[4 * WL];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const int dxl = l >> 5, cl = l & 31;
  const long long nrays = (long long)a.B * a.HW;
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= nrays) return;
  float* X = lds + wv * WL;
  float* Mt = X + XTILE;
  const bool dcoord = g.g_ro != nullptr;

  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};
  float* __restrict__ dpl = g.d_planes + (long long)R.b * a.field.sb;
  const float* pal = a.field.palette + R.b * (NA * 3);

  const float gr0 = g.g_rgb[r * 3 + 0], gr1 = g.g_rgb[r * 3 + 1], gr2 = g.g_rgb[r * 3 + 2];
  const float gm = g.g_mask[r] - (a.white_bg ? (gr0 + gr1 + gr2) : 0.f);

  // ---- compositing backward ----
  float t[NPL], sg[NPL], al[NPL], aa[NPL], ex[NPL], dist[NPL], raw[NPL], T[NPL], ee[NPL];
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    t[e] = (i < N) ? a.t_saved[r * N + i] : 0.f;
    Mt[e * 64 + l] = t[e];
  }
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    const bool v = i < N;
    sg[e] = v ? a.sigma_saved[r * N + i] : 0.f;
    raw[e] = (i < N - 1) ? (Mt[i + 1] - t[e]) : 0.f;
    dist[e] = raw[e] * R.rdn;
    ex[e] = expf(-sg[e] * dist[e]);
    al[e] = v ? 1.f - ex[e] : 0.f;
    aa[e] = v ? (1.f - al[e]) + 1e-10f : 1.f;
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;
    if (v) {
      c0 = a.rgb_saved[(r * 3 + 0) * N + i];
      c1 = a.rgb_saved[(r * 3 + 1) * N + i];
      c2 = a.rgb_saved[(r * 3 + 2) * N + i];
    }
    ee[e] = v ? (gr0 * c0 + gr1 * c1 + gr2 * c2) + gm : 0.f;
  }
  excl_prod<NPL>(aa, T);
  // S_k = sum_{i>k} e_i alpha_i prod_{k<j<i} a_j  : reverse exclusive scan of f_i(s) = a_i s + e_i alpha_i
  float gsig[NPL], gcw[NPL];
  float grdn = 0.f;
  {
    float cA = 1.f, cB = 0.f;   // composition of maps with index beyond the current chunk
#pragma unroll
    for (int e = NPL - 1; e >= 0; --e) {
      float A = aa[e], B = ee[e] * al[e];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const float A2 = __shfl_down(A, d), B2 = __shfl_down(B, d);
        if (l + d < 64) {
          B = fmaf(A, B2, B);
          A = A * A2;
        }
      }
      // exclusive: F_{l+1} o carry evaluated at 0
      float An = __shfl_down(A, 1), Bn = __shfl_down(B, 1);
      float Sk = (l < 63) ? fmaf(An, cB, Bn) : cB;
      const float A0 = readlane(A, 0), B0 = readlane(B, 0);
      cB = fmaf(A0, cB, B0);
      cA = A0 * cA;
      const float dal = T[e] * (ee[e] - Sk);
      gsig[e] = dal * dist[e] * ex[e];
      grdn += dal * sg[e] * ex[e] * raw[e];
      gcw[e] = al[e] * T[e];   // weight w_i; d c_i = w_i * g_rgb
    }
  }

  // ---- per-sample field backward ----
  float gro[3] = {0.f, 0.f, 0.f}, grd[3] = {0.f, 0.f, 0.f};
  float dpal[NA * 3];
#pragma unroll
  for (int k = 0; k < NA * 3; ++k) dpal[k] = 0.f;

#pragma unroll 1
  for (int e = 0; e < NPL; ++e) {
    const int npts = min(64, N - e * 64);
    const int i = e * 64 + l;
    const bool v = i < N;
    PointP P;
    point_params(R.o, R.d, t[e], a.field.scene_range, pv.R, P);
    gather_features(pv, P, npts, X);
    wave_lds_sync();
    float x[NC];
    load_row(X, l, x);
    float y[NO];
    mlp_forward(a.field.dec, x, y);
    Head h;
    head_forward(y, P.mask, a.field.inv_alpha, a.field.beta, pal, h);
    // sigma -> distance
    const float gs = v ? gsig[e] : 0.f;
    const float xn = -y[0];
    const float sgn = tsign(xn);
    const float ex2 = expf(-fabsf(xn) / a.field.beta);
    const float gcdf = (gs * a.field.inv_alpha) * (1.f - P.mask);
    const float gxn = ((gcdf * 0.5f * sgn) * ex2 / a.field.beta) * sgn;
    float gy[NO];
    gy[0] = -gxn;
    // rgb -> logits (softmax backward), palette gradient
    const float w = v ? gcw[e] : 0.f;
    const float gc0 = w * gr0, gc1 = w * gr1, gc2 = w * gr2;
    float gp[NA], dot = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      gp[k] = gc0 * pal[k * 3 + 0] + gc1 * pal[k * 3 + 1] + gc2 * pal[k * 3 + 2];
      dot = fmaf(gp[k], h.p[k], dot);
      dpal[k * 3 + 0] = fmaf(h.p[k], gc0, dpal[k * 3 + 0]);
      dpal[k * 3 + 1] = fmaf(h.p[k], gc1, dpal[k * 3 + 1]);
      dpal[k * 3 + 2] = fmaf(h.p[k], gc2, dpal[k * 3 + 2]);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) gy[1 + k] = (gp[k] - dot) * h.p[k];
    float gx[NC];
    mlp_backward(a.field.dec, x, gy, gx);
#pragma unroll
    for (int c = 0; c < NC; ++c) gx[c] = gx[c] / 3.f;   // x = (e1+e2+e3)/3
    wave_lds_sync();
    store_row(X, l, gx);
    wave_lds_sync();
    // scatter-add d planes (+ re-gather for d coords), one point at a time, 256-B rows
#pragma unroll 1
    for (int j = 0; j < npts; ++j) {
      const float gv = X[j * XS + cl];
      float GX[3], GY[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int pk = readlane(P.pl[q].tex, j);
        const float ew = readlane(P.pl[q].e, j), ww = readlane(P.pl[q].w, j);
        const float s = readlane(P.pl[q].s, j), n = readlane(P.pl[q].n, j);
        const int t0 = (pk & 0xFFFFF) + (dxl ? ((pk >> 20) & 1) : 0);
        const int t1 = t0 + (((pk >> 21) & 1) ? pv.R : 0);
        const float wx = dxl ? ww : ew;
        float* dq = dpl + q * pv.sq + cl;
        unsafeAtomicAdd(dq + t0 * pv.st, gv * (s * wx));
        unsafeAtomicAdd(dq + t1 * pv.st, gv * (n * wx));
        if (dcoord) {
          const float* bq = pv.base + q * pv.sq + cl;
          const float v0 = bq[t0 * pv.st], v1 = bq[t1 * pv.st];
          const float px = (dxl ? 1.f : -1.f) * (s * v0 + n * v1) * gv;
          const float py = wx * (v1 - v0) * gv;
          GX[q] = wave_sum(px) * readlane(P.pl[q].gxm, j);
          GY[q] = wave_sum(py) * readlane(P.pl[q].gym, j);
        }
      }
      if (dcoord) {
        const float tj = readlane(t[e], j);
        const float sr = a.field.scene_range;
        const float dp0 = (GX[0] + GX[1]) / sr;
        const float dp1 = (GY[0] + GX[2]) / sr;
        const float dp2 = (GY[1] + GY[2]) / sr;
        gro[0] += dp0;
        gro[1] += dp1;
        gro[2] += dp2;
        grd[0] = fmaf(dp0, tj, grd[0]);
        grd[1] = fmaf(dp1, tj, grd[1]);
        grd[2] = fmaf(dp2, tj, grd[2]);
      }
    }
    wave_lds_sync();
  }

  // ---- per-ray outputs ----
#pragma unroll
  for (int k = 0; k < NA * 3; ++k) {
    const float s = wave_sum(dpal[k]);
    if (l == 0) g.d_palette_ray[r * (NA * 3) + k] = s;
  }
  if (dcoord) {
    grdn = wave_sum(grdn);
    if (l == 0) {
      // dists * ||rd||  ->  d rd += d||rd|| * rd / ||rd||
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        g.g_ro[r * 3 + k] = gro[k];
        g.g_rd[r * 3 + k] = grd[k] + grdn * (R.d[k] / R.rdn);
      }
    }
  }
}

template <int S, bool FINE>
static int launch_pair(const nfi_render_args* a, const nfi_render_grad_args* g, hipStream_t s) {
  const long long nrays = (long long)a->B * a->HW;
  const unsigned blocks = (unsigned)((nrays + 3) / 4);
  if (g == nullptr) {
    render_fwd_kernel<S, FINE><<<blocks, 256, 0, s>>>(*a);
    NFI_CHECK_LAUNCH("render_fwd_kernel");
  } else {
    render_bwd_kernel<S, FINE><<<blocks, 256, 0, s>>>(*a, *g);
    NFI_CHECK_LAUNCH("render_bwd_kernel");
  }
  return NFI_OK;
}

static int dispatch(const nfi_render_args* a, const nfi_render_grad_args* g, hipStream_t s) {
  const bool f = a->fine != 0;
  switch (a->S) {
    case 32: return f ? launch_pair<32, true>(a, g, s) : launch_pair<32, false>(a, g, s);
    case 64: return f ? launch_pair<64, true>(a, g, s) : launch_pair<64, false>(a, g, s);
    case 128: return f ? launch_pair<128, true>(a, g, s) : launch_pair<128, false>(a, g, s);
    case 256:
      if (!f) return launch_pair<256, false>(a, g, s);
      break;
    default: break;
  }
  set_error("render: unsupported samples per ray S=%d (fine=%d)", a->S, (int)f);
  return NFI_EINVAL;
}

static int validate(const nfi_render_args* a) {
  NFI_REQUIRE(a != nullptr, "render: null args");
  const nfi_field& f = a->field;
  NFI_REQUIRE(f.planes && f.dec && f.palette, "render: null field pointer");
  NFI_REQUIRE(f.R >= 2 && f.R <= 1024, "render: plane resolution R=%d out of range [2,1024]", f.R);
  NFI_REQUIRE(f.st >= NC && 3LL * f.sq < (1LL << 31) && (long long)f.R * f.R * f.st < (1LL << 31),
              "render: plane strides out of range (st=%lld sq=%lld)", (long long)f.st, (long long)f.sq);
  NFI_REQUIRE(f.beta > 0.f && std::isfinite(f.inv_alpha) && f.scene_range > 0.f, "render: bad field scalars");
  NFI_REQUIRE(a->ro && a->rd && a->near_ && a->far_, "render: null ray pointer");
  NFI_REQUIRE(a->B > 0 && a->HW > 0, "render: bad shape B=%d HW=%d", a->B, a->HW);
  NFI_REQUIRE(a->t_saved && a->sigma_saved && a->rgb_saved, "render: null saved-state pointer");
  return NFI_OK;
}

}  // namespace nfi

extern "C" {

int32_t nfi_render_forward(const nfi_render_args* a, void* stream) {
  int e = nfi::validate(a);
  if (e) return e;
  NFI_REQUIRE(a->rgb && a->depth && a->mask, "render_forward: null output");
  return nfi::dispatch(a, nullptr, (hipStream_t)stream);
}

int32_t nfi_render_backward(const nfi_render_args* a, const nfi_render_grad_args* g, void* stream) {
  int e = nfi::validate(a);
  if (e) return e;
  NFI_REQUIRE(g && g->g_rgb && g->g_mask && g->d_planes && g->d_palette_ray, "render_backward: null grad pointer");
  NFI_REQUIRE((g->g_ro == nullptr) == (g->g_rd == nullptr), "render_backward: g_ro/g_rd must both be set or null");
  return nfi::dispatch(a, g, (hipStream_t)stream);
}

}  // extern "C"
