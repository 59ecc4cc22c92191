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
#include <cstdlib>
#include <cstring>

#include "nfi_common.h"
#include "nfi_host.h"

namespace nfi {

#ifdef NFI_STAMPS
__device__ unsigned long long nfi_stamp_acc[STAMP_SLOTS * STAMP_PHASES];
#endif

constexpr int XS = 36;                  // LDS row stride (floats) of the point x channel tile
constexpr int XTILE = WAVE * XS;        // 2304 floats

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// N floats (dst 16-byte aligned) to LDS as b128 stores (the tail b64 / b32), each followed by the 2 wait
// states of lds_st (nfi_common.h).  (Round 3 used 32-bit stores + s_waitcnt lgkmcnt(0) here, for
// the same hazard: DESIGN.md §3.)
template <int N>
__device__ __forceinline__ void lds_store_keep(float* __restrict__ dst, const float (&v)[N]) {
#if !NFI_LDS_GAP
  volatile float* d = dst;   // round 3: 32-bit stores, then lgkmcnt(0) and an empty use of every value
#pragma unroll
  for (int k = 0; k < N; ++k) d[k] = v[k];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" ::"v"(v[k]));
  return;
#endif
#pragma unroll
  for (int k = 0; k + 4 <= N; k += 4)
    lds_st(reinterpret_cast<float4*>(dst + k), make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]));
  if constexpr (N % 4 >= 2) lds_st(reinterpret_cast<float2*>(dst + N / 4 * 4), make_float2(v[N / 4 * 4], v[N / 4 * 4 + 1]));
  if constexpr (N % 2 == 1) dst[N - 1] = v[N - 1];
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
  // ray_origins + ray_directions * depth (run.py:283-288, nerf_utils.py:121), then / scene_range
  // (generator.py:604): two roundings each, as ATen evaluates them.
#pragma unroll
  for (int k = 0; k < 3; ++k) P.cx[k] = fdiv(fadd(o[k], fmul(d[k], t)), sr);
  P.mask = (fabsf(P.cx[0]) > 1.f || fabsf(P.cx[1]) > 1.f || fabsf(P.cx[2]) > 1.f) ? 1.f : 0.f;
  plane_params(P.cx[0], P.cx[1], R, P.pl[0]);
  plane_params(P.cx[0], P.cx[2], R, P.pl[1]);
  plane_params(P.cx[1], P.cx[2], R, P.pl[2]);
}

struct PlaneView {
  const float* __restrict__ base;   // planes of this image
  int sq, st, R;
};

// Gather + interpolate + mean-of-3 for points 0..npts-1 of the wave; writes X[j][0..31]
// (j < npts) into the wave's LDS tile.
//
// Lane layout ("quad" gather): lane = (sub = l>>4, dx = (l>>3)&1, q4 = l&7).  One wave
// instruction serves four points (sub), each a bilinear row pair of 2 texels x 32 channels
// (dx selects x0 / x0+1, q4 a float4 of channels): 4 x 256 contiguous bytes per 1-KiB load,
// through a buffer resource on the image's planes (no per-load 64-bit address arithmetic).
// The three planes' weighted texels are summed per lane before the one DPP row_ror:8 that adds
// the x0 / x0+1 lanes (the bilinear tap and the plane mean are both linear).
//
// Load records: every lane first writes its own point's records into its row of the X tile —
// per (plane, dx) the byte offsets of the two texel rows and their two weights with the mean's
// 1/3 folded in, {t0, t1, W0/3, W1/3} — and a lane serving point j fetches its record with one
// ds_read_b128 per plane.  The records of row j are read when group j/4 is issued; the row is
// overwritten by that group's features only after (a wave's LDS operations complete in order).
// Measured on MI355X (render_fwd, p3d B=8): 2.24 ms against 2.27-2.32 ms for the same gather
// with the parameters ds_bpermuted from the owning lane and unpacked per serving lane and group
// (~40 more VALU per group).  Variants that did not pay: a software pipeline over single groups
// (2.58 vs 2.50 ms, r02), 3-4 groups per batch (spills at the occupancy-4 register budget),
// dword prefetches of the next batch's lines (2.93 ms: the gather is bound by the texture
// path's request rate, which the extra requests share, not by latency alone).
__device__ __forceinline__ float4 ror8_add(float4 v) {
  v.x += dpp_mov<0x128>(v.x);
  v.y += dpp_mov<0x128>(v.y);
  v.z += dpp_mov<0x128>(v.z);
  v.w += dpp_mov<0x128>(v.w);
  return v;
}

// Loads of GB groups (4*GB points) are issued before any is consumed (6*GB KiB in flight per wave).
#ifndef NFI_GATHER_GB
#define NFI_GATHER_GB 2
#endif
constexpr int GATHER_GB = NFI_GATHER_GB;

__device__ __forceinline__ void gather_records(const PlaneView& pv, const PointP& P, float* __restrict__ X) {
  const int st4 = pv.st * 4, rowb = pv.R * pv.st * 4, sq4 = pv.sq * 4;
  float* row = X + lane_id() * XS;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int t = P.pl[q].tex;
    const int o0 = (t & 0xFFFFF) * st4 + q * sq4;
    const int o1 = o0 + (((t >> 20) & 1) ? st4 : 0);
    const int dy = ((t >> 21) & 1) ? rowb : 0;
    const float w = P.pl[q].w, n = P.pl[q].n, e = 1.f - w, s = 1.f - n;
    // record (weight row 0, offset row 0, weight row 1, offset row 1): the weights land in even
    // registers of the b128 read, where the packed interpolation takes them as aligned pairs (with
    // (offset, offset, weight, weight) the odd-register weight took a v_mov per plane and group)
    lds_st(reinterpret_cast<float4*>(row + 8 * q),
           make_float4((s * e) * (1.f / 3.f), __int_as_float(o0), (n * e) * (1.f / 3.f), __int_as_float(o0 + dy)));
    lds_st(reinterpret_cast<float4*>(row + 8 * q + 4),
           make_float4((s * w) * (1.f / 3.f), __int_as_float(o1), (n * w) * (1.f / 3.f), __int_as_float(o1 + dy)));
  }
}

__device__ __forceinline__ void gather_issue(__amdgpu_buffer_rsrc_t rsrc, const float* __restrict__ X, int g,
                                              int sub, int dx, int q4, float4 (&V0)[3], float4 (&V1)[3],
                                              float (&W0)[3], float (&W1)[3]) {
  const float* rec = X + (4 * g + sub) * XS + 4 * dx;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float4 R = *reinterpret_cast<const float4*>(rec + 8 * q);
    const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, __float_as_int(R.y) + 16 * q4, 0, 0);
    const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, __float_as_int(R.w) + 16 * q4, 0, 0);
    V0[q] = make_float4(__int_as_float(v0[0]), __int_as_float(v0[1]), __int_as_float(v0[2]), __int_as_float(v0[3]));
    V1[q] = make_float4(__int_as_float(v1[0]), __int_as_float(v1[1]), __int_as_float(v1[2]), __int_as_float(v1[3]));
    W0[q] = R.x;
    W1[q] = R.z;
  }
}

__device__ __forceinline__ void gather_consume(int g, int sub, int dx, int q4, int npts, const float4 (&V0)[3],
                                                const float4 (&V1)[3], const float (&W0)[3],
                                                const float (&W1)[3], float* __restrict__ X) {
  const int j = 4 * g + sub;
  float4 pr;
  pr.x = (V0[0].x * W0[0] + V1[0].x * W1[0]) + (V0[1].x * W0[1] + V1[1].x * W1[1]) + (V0[2].x * W0[2] + V1[2].x * W1[2]);
  pr.y = (V0[0].y * W0[0] + V1[0].y * W1[0]) + (V0[1].y * W0[1] + V1[1].y * W1[1]) + (V0[2].y * W0[2] + V1[2].y * W1[2]);
  pr.z = (V0[0].z * W0[0] + V1[0].z * W1[0]) + (V0[1].z * W0[1] + V1[1].z * W1[1]) + (V0[2].z * W0[2] + V1[2].z * W1[2]);
  pr.w = (V0[0].w * W0[0] + V1[0].w * W1[0]) + (V0[1].w * W0[1] + V1[1].w * W1[1]) + (V0[2].w * W0[2] + V1[2].w * W1[2]);
  const float4 E = ror8_add(pr);
  if (dx == 0 && j < npts) *reinterpret_cast<float4*>(X + j * XS + 4 * q4) = E;
}

__device__ __forceinline__ void gather_features(const PlaneView& pv, const PointP& P, int npts,
                                                float* __restrict__ X) {
  const int l = lane_id();
  const int sub = l >> 4, dx = (l >> 3) & 1, q4 = l & 7;
  const int ngrp = (npts + 3) >> 2;
  gather_records(pv, P, X);
  wave_lds_sync();
  const uint64_t pb = reinterpret_cast<uint64_t>(pv.base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pb >> 32));
  // the resource spans exactly this image's three planes (last texel's last channel + 1): a load
  // at any offset past them returns zeros instead of touching memory
  const int extent = __builtin_amdgcn_readfirstlane(((pv.R * pv.R - 1) * pv.st + 2 * pv.sq + NC) * 4);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, extent, 0x00020000);
#pragma unroll 1
  for (int gb = 0; gb < ngrp; gb += GATHER_GB) {
    float4 V0[GATHER_GB][3], V1[GATHER_GB][3];
    float W0[GATHER_GB][3], W1[GATHER_GB][3];
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) gather_issue(rsrc, X, gb + u, sub, dx, q4, V0[u], V1[u], W0[u], W1[u]);
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) gather_consume(gb + u, sub, dx, q4, npts, V0[u], V1[u], W0[u], W1[u], X);
  }
}

// ---------------------------------------------------------------------------------------
// d planes by plane tile: every (sample, plane) contribution is binned by the 7x4-cell tile of
// the plane its bilinear cell lies in, and a workgroup sums a chunk of one tile's entries in
// REGISTERS: lane (h, c) of a wave holds channel c of texel rows ly + h of the tile's 8x5 texels
// as a 32-float vector (half h = 1 stores row y at slot y - 1, so an entry's two rows sit at the
// same wave-uniform slot ly*8 + lx in both halves), updated through a wave-uniform jump table of
// static-register FMAs (tile_entry).  No LDS atomics (gfx950 ds_add_f32: ~200 cycles per wave-instruction per CU)
// and no LDS read-modify-write chain; the waves' images are merged once through LDS and flushed
// with one global float atomic per nonzero texel channel.
//
// Cells are normalized so the bilinear cell is interior (x0, y0 <= R-2): a border-clipped point
// (x0 = R-1, w = 0) becomes (x0 = R-2, w = 1), which puts the same weights on the same texels.
// ---------------------------------------------------------------------------------------
constexpr int TSX = 7, TSY = 4;               // cells per tile
constexpr int TTX = TSX + 1, TTY = TSY + 1;   // texels per tile (8 x 5)
#ifndef NFI_TILE_CHUNK
#define NFI_TILE_CHUNK 2048   // 1024 / 4096 measured within noise (2.23-2.35 ms)
#endif
constexpr int CHUNK = NFI_TILE_CHUNK;         // (sample, plane) entries per accumulation workgroup

// Ray blocks ("beams"): every image's pixels are split into sx x sy rectangles and the bins are
// keyed per (beam, plane, tile), so the tile pass works through the batch beam by beam.  A beam's
// samples have their three (plane, tile) entries in three different tiles; keyed per image, the
// three reads of one sample's 128-B gradient row were a third of an image's entries apart (HBM
// each time: B=8 reads 6.4 GB of rows per launch); keyed per beam of ~NFI_BEAM_SAMPLES samples
// (rows + records ~90 MB at 2^19) the second and third reads fall inside one beam's window and hit
// the 256 MB Infinity Cache.  0 = one beam per image (the per-image keys).
#ifndef NFI_BEAM_SAMPLES
#define NFI_BEAM_SAMPLES 0
#endif
struct TileGrid {
  int nx, ny;   // plane tiles
  int sx, sy;   // beams per image: sx columns x sy rows of pixels
  int W, H;     // image (H = 0: one beam per image)
};
__host__ __device__ __forceinline__ TileGrid tile_grid(int R, int HW = 0, int W = 0, int N = 0) {
  TileGrid g{(R - 2) / TSX + 1, (R - 2) / TSY + 1, 1, 1, W, 0};
  if (NFI_BEAM_SAMPLES > 0 && W > 0 && HW % W == 0 && N > 0) {
    g.H = HW / W;
    // halve the longer side of the beam while a beam holds more than NFI_BEAM_SAMPLES samples
    while ((long long)HW * N / (g.sx * g.sy) > NFI_BEAM_SAMPLES && g.sx * g.sy < 64) {
      if (W / g.sx >= g.H / g.sy && W / g.sx >= 32) g.sx *= 2;
      else if (g.H / g.sy >= 32) g.sy *= 2;
      else break;
    }
  }
  return g;
}
__host__ __device__ __forceinline__ int beams_per_image(TileGrid G) { return G.sx * G.sy; }
// beam index of ray r (of B*HW, images HW = H*W pixels apart, row-major pixels)
__device__ __forceinline__ int beam_of(long long r, int HW, TileGrid G) {
  const int b = (int)(r / HW);
  if (G.sx * G.sy == 1) return b;
  const int p = (int)(r - (long long)b * HW), row = p / G.W, col = p - row * G.W;
  return b * (G.sx * G.sy) + (row * G.sy / G.H) * G.sx + col * G.sx / G.W;
}

// Tile keys order the accumulation chunks: beam-major (above), then per beam the x-slabs tx with
// the xy tiles (tx, y) and the xz tiles (tx, z) of a slab next to each other, followed by the yz
// tiles.
__host__ __device__ __forceinline__ int tile_key(int beam, int q, int tx, int ty, TileGrid G) {
  const int T = G.nx * G.ny;
  return beam * 3 * T + (q == 2 ? 2 * T + ty * G.nx + tx : (tx * 2 + q) * G.ny + ty);
}
// b = the IMAGE of the key's beam
__device__ __forceinline__ void tile_decode(int key, TileGrid G, int& b, int& q, int& tx, int& ty) {
  const int T = G.nx * G.ny;
  b = key / (3 * T) / beams_per_image(G);
  const int r = key % (3 * T);
  if (r >= 2 * T) {
    q = 2;
    ty = (r - 2 * T) / G.nx;
    tx = (r - 2 * T) % G.nx;
  } else {
    tx = r / (2 * G.ny);
    q = (r / G.ny) & 1;
    ty = r % G.ny;
  }
}

// Tile key of plane q for point P of beam `beam` (beam_of), and the entry record {s, slot | flags, w, n}:
// slot = ly*8 + lx inside the tile, flags bit 8/9 = grid-gradient multiplier gxm/gym nonzero.
__device__ __forceinline__ int plane_tile_key(const PointP& P, int q, int b, int R, TileGrid G, long long s,
                                              int4& rec) {
  const int cell = P.pl[q].tex & 0xFFFFF;
  int y0 = cell / R, x0 = cell % R;
  float w = P.pl[q].w, n = P.pl[q].n;
  if (x0 == R - 1) {
    x0 = R - 2;
    w = 1.f;
  }
  if (y0 == R - 1) {
    y0 = R - 2;
    n = 1.f;
  }
  const int tx = x0 / TSX, ty = y0 / TSY;
  const int slot = (y0 - ty * TSY) * TTX + (x0 - tx * TSX);
  rec = make_int4((int)s, slot | (P.pl[q].gxm != 0.f ? 0x100 : 0) | (P.pl[q].gym != 0.f ? 0x200 : 0),
                  __float_as_int(w), __float_as_int(n));
  return tile_key(b, q, tx, ty, G);
}

// Run-aggregated atomicAdd of 1 per valid lane on base[key]: each run of equal keys in
// consecutive lanes (samples along a ray are depth-sorted, so a ray meets each tile in one run)
// takes its slots with ONE atomic by the run's first lane, all runs in one wave instruction —
// one memory round trip per call whatever the key pattern (a key split over several runs gets
// one contiguous slot range per run).  Returns each lane's slot.
struct LaneRuns {
  int leader;   // first lane of this lane's run
  int len;      // run length (meaningful in leader lanes)
  bool start;
};
__device__ __forceinline__ LaneRuns lane_runs(int key, bool valid) {
  const int l = lane_id();
  const int kk = valid ? key : -1;
  const int prev = __shfl_up(kk, 1);
  LaneRuns R;
  R.start = (l == 0) || kk != prev;
  const unsigned long long starts = __ballot(R.start);
  const unsigned long long upto = (l == 63) ? ~0ull : ((2ull << l) - 1ull);   // lanes <= l
  R.leader = 63 - __clzll(starts & upto);
  const unsigned long long after = starts & ~upto;
  R.len = (after ? (__ffsll((long long)after) - 1) : 64) - l;
  return R;
}
__device__ __forceinline__ int run_increment(int* base, int key, bool valid) {
  const LaneRuns R = lane_runs(key, valid);
  int old = 0;
  if (R.start && valid) old = atomicAdd(base + key, R.len);
  return __shfl(old, R.leader) + (lane_id() - R.leader);
}
__device__ __forceinline__ void run_count(int* base, int key, bool valid) {
  const LaneRuns R = lane_runs(key, valid);
  if (R.start && valid) atomicAdd(base + key, R.len);
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

// Softplus(beta=1, threshold=20) (generator.py:297) and its derivative (ATen softplus_backward)
// on the transcendental units: log(1 + e^z) = log2(1 + 2^(z log2 e)) ln 2.  Rounding 1 + e^z
// costs at most 2^-24 ABSOLUTE in the result (log' <= 1 near 1), the size of an fp32 rounding
// of the O(1) hidden activations it feeds, so the log1p correction is not carried.
// sigmoid(z) = 1 / (1 + e^-z) is exactly 1 in fp32 beyond the threshold and 0 far below it.
__device__ __forceinline__ float softplus(float z) {
  const float u = __builtin_amdgcn_exp2f(z * 1.44269504f);
  const float h = __builtin_amdgcn_logf(1.f + u) * 0.69314718f;
  return (z > 20.f) ? z : h;
}
__device__ __forceinline__ float softplus_grad(float z) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z * -1.44269504f));
}
// the same from z' = z log2(e) (the DT1S / DB1S tables): one multiply fewer per hidden unit in
// the field backward, which is bound by the SIMD datapath
__device__ __forceinline__ float softplus_grad2(float zs) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-zs));
}
#ifndef NFI_SP2B
#define NFI_SP2B 1
#endif

// ---------------------------------------------------------------------------------------
// Decoder on the matrix cores: v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fmaf chain per
// output) for the 64 points of a wave, in the orientation that lets each product's result feed
// the next one straight from its accumulator registers (operand tables: nfi_common.h DT*).
// Points are columns: block sb holds points 16sb..16sb+15; lane l = (j = l&15, q = l>>4).
//   Z^T  [64 hid x 64 pts] = W1s X^T + b1        A = DT1, B = X^T (lane: point j, channels 8q+t)
//   Y^T  [11 out x 64 pts] = W2s softplus(Z)^T   B = softplus(Z) accumulator registers
//   dH^T [64 x 64]         = W2s^T dY^T          A = DT3, B = dY^T (through LDS)
//   dX^T [32 x 64]         = W1s^T (dH o sigmoid(Z))^T   B = accumulator registers
// The VALU is left with softplus / sigmoid and the surrounding per-point work.
// ---------------------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v ld4(const float* p) { return *reinterpret_cast<const f4v*>(p); }
// The forward's saved decoder inputs / outputs (2.8 GB per B=8 launch, read once by the field
// backward) are written with the nontemporal hint, so they do not evict the plane texels the
// gathers re-read from L2 / the Infinity Cache (forward ~1 % faster).  The same hint on the field
// backward's x loads and feature-gradient stores measured 4 % slower there.  NFI_NT 0: off.
#ifndef NFI_NT
#define NFI_NT 1
#endif
__device__ __forceinline__ void nt_store4(float4* p, float4 v) {
#if NFI_NT
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
#else
  *p = v;
#endif
}
#if NFI_NT
#define NFI_NT_STORE(P, V) __builtin_nontemporal_store((V), (P))
#else
#define NFI_NT_STORE(P, V) (*(P) = (V))
#endif
__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Z^T block (hb, sb) = W1s[16hb.., :] X^T[:, 16sb..] + b1: xa/xb = channels 8q..8q+3, 8q+4..8q+7
// of point 16sb + j; ta/tb = DT1 k-steps 0..3, 4..7; b = DB1
__device__ __forceinline__ f4v layer1(f4v ta, f4v tb, f4v b, f4v xa, f4v xb) {
  f4v z = b;
  z = mfma4(ta[0], xa[0], z);
  z = mfma4(ta[1], xa[1], z);
  z = mfma4(ta[2], xa[2], z);
  z = mfma4(ta[3], xa[3], z);
  z = mfma4(tb[0], xb[0], z);
  z = mfma4(tb[1], xb[1], z);
  z = mfma4(tb[2], xb[2], z);
  z = mfma4(tb[3], xb[3], z);
  return z;
}

// Decoder forward for the points of the wave's X tile (LDS, rows of XS floats); returns point
// l's NOUT outputs.  The tile is reused as scratch (callers re-sync before writing it).
template <int NOUT, bool PREFETCH>
__device__ __forceinline__ void mlp_forward_tile(const float* __restrict__ dec, float* __restrict__ X,
                                                 float y[NOUT]) {
  using L = DecL<NOUT>;
  constexpr int NOB = L::NOB;
  const int l = lane_id(), j = l & 15, q = l >> 4;
  f4v xa[4], xb[4];
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    xa[sb] = ld4(X + (16 * sb + j) * XS + 8 * q);
    xb[sb] = ld4(X + (16 * sb + j) * XS + 8 * q + 4);
  }
  f4v Y[NOB][4];
#pragma unroll
  for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) Y[ob][sb] = f4v{0.f, 0.f, 0.f, 0.f};
  if constexpr (PREFETCH) {
  // operand tables of hidden block hb + 1 are loaded while block hb runs (L1/L2 round trips
  // otherwise serialise with the MFMA chains: 16 more VGPRs — used by the occupancy-2 kernels;
  // the inversion forward runs at occupancy 4 without them, render_fwd_kernel)
  f4v ta = ld4(dec + L::DT1 + l * 8), tb = ld4(dec + L::DT1 + l * 8 + 4);
  f4v b = ld4(dec + L::DB1 + l * 4);
  f4v t2[NOB];
#pragma unroll
  for (int ob = 0; ob < NOB; ++ob) t2[ob] = ld4(dec + L::DT2 + (ob * 256 + l) * 4);
#pragma unroll
  for (int hb = 0; hb < 4; ++hb) {
    f4v nta = ta, ntb = tb, nb = b, nt2[NOB];
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob) nt2[ob] = t2[ob];
    if (hb < 3) {
      const int hn = hb + 1;
      nta = ld4(dec + L::DT1 + (hn * 64 + l) * 8);
      ntb = ld4(dec + L::DT1 + (hn * 64 + l) * 8 + 4);
      nb = ld4(dec + L::DB1 + (hn * 64 + l) * 4);
#pragma unroll
      for (int ob = 0; ob < NOB; ++ob) nt2[ob] = ld4(dec + L::DT2 + ((ob * 4 + hn) * 64 + l) * 4);
    }
    __builtin_amdgcn_sched_barrier(0);   // (keeps the scheduler from sinking the loads to their use)
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const f4v z = layer1(ta, tb, b, xa[sb], xb[sb]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sp = softplus(z[r]);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) Y[ob][sb] = mfma4(t2[ob][r], sp, Y[ob][sb]);
      }
    }
    ta = nta;
    tb = ntb;
    b = nb;
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob) t2[ob] = nt2[ob];
  }
  } else {
#pragma unroll
  for (int hb = 0; hb < 4; ++hb) {
    const f4v ta = ld4(dec + L::DT1 + (hb * 64 + l) * 8), tb = ld4(dec + L::DT1 + (hb * 64 + l) * 8 + 4);
    const f4v b = ld4(dec + L::DB1 + (hb * 64 + l) * 4);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const f4v z = layer1(ta, tb, b, xa[sb], xb[sb]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sp = softplus(z[r]);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
          Y[ob][sb] = mfma4(ld4(dec + L::DT2 + ((ob * 4 + hb) * 64 + l) * 4)[r], sp, Y[ob][sb]);
      }
    }
  }
  }
  // lane (j, q) holds outputs 16ob + 4q..4q+3 of point 16sb + j: transpose through the tile
  // (outputs past NOUT's last quad are not stored: 33 outputs use columns 0..35 of the XS = 36 row)
  wave_lds_sync();
#pragma unroll
  for (int sb = 0; sb < 4; ++sb)
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob)
      if (16 * NOB <= XS || ob + 1 < NOB || 16 * ob + 4 * q < NOUT)
        *reinterpret_cast<f4v*>(X + (16 * sb + j) * XS + 16 * ob + 4 * q) = Y[ob][sb];
  wave_lds_sync();
#pragma unroll
  for (int o = 0; o < NOUT; ++o) y[o] = X[l * XS + o] + dec[L::DB2 + o];
}
static_assert(4 * DecL<NOV>::KT <= XS, "33 decoder outputs fit an X tile row");

// Decoder input-gradient (weights frozen during inversion, run.py:630-632) for 64 points:
// xa/xb as layer1's operands for blocks sb; dY^T operands gyb[sb][t] = dY[16sb + j][4t + q];
// returns dX^T accumulators gxo[cb][sb] (lane: channels 16cb + 4q + reg of point 16sb + j).
template <int NOUT>
__device__ __forceinline__ void mlp_backward_mfma(const float* __restrict__ dec, const f4v xa[4], const f4v xb[4],
                                                  const float gyb[4][DecL<NOUT>::KT], f4v gxo[2][4]) {
  using L = DecL<NOUT>;
  const int l = lane_id();
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) gxo[cb][sb] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int hb = 0; hb < 4; ++hb) {
#if NFI_SP2B
    const f4v ta = ld4(dec + L::DT1S + (hb * 64 + l) * 8), tb = ld4(dec + L::DT1S + (hb * 64 + l) * 8 + 4);
    const f4v b = ld4(dec + L::DB1S + (hb * 64 + l) * 4);
#else
    const f4v ta = ld4(dec + L::DT1 + (hb * 64 + l) * 8), tb = ld4(dec + L::DT1 + (hb * 64 + l) * 8 + 4);
    const f4v b = ld4(dec + L::DB1 + (hb * 64 + l) * 4);
#endif
    f4v t3[L::KTP / 4];
#pragma unroll
    for (int u = 0; u < L::KTP / 4; ++u) t3[u] = ld4(dec + L::DT3 + (hb * 64 + l) * L::KTP + 4 * u);
    const f4v t40 = ld4(dec + L::DT4 + ((0 * 4 + hb) * 64 + l) * 4);
    const f4v t41 = ld4(dec + L::DT4 + ((1 * 4 + hb) * 64 + l) * 4);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const f4v z = layer1(ta, tb, b, xa[sb], xb[sb]);
      f4v gh = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < L::KT; ++t) gh = mfma4(t3[t >> 2][t & 3], gyb[sb][t], gh);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#if NFI_SP2B
        const float gz = gh[r] * softplus_grad2(z[r]);
#else
        const float gz = gh[r] * softplus_grad(z[r]);
#endif
        gxo[0][sb] = mfma4(t40[r], gz, gxo[0][sb]);
        gxo[1][sb] = mfma4(t41[r], gz, gxo[1][sb]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// The inversion decoder (11 outputs) on the f16 matrix cores at fp32 accuracy.
// v_mfma_f32_16x16x32_f16 runs a 16x16x32 product in 16 cycles, v_mfma_f32_16x16x4_f32 a 16x16x4
// in 32: per unit of K the f16 form is 16x the f32 one.  Every fp32 operand v (scaled by a power
// of two, exact) is carried as hi = f16(v), lo = f16(v - hi) (round-to-nearest: v = hi + lo to
// 2^-22 |v| at worst, 2^-24 typically), and a contraction is lo.hi + hi.lo + hi.hi on one fp32
// accumulator — the dropped lo.lo term is below an fp32 rounding of the product.  Products of f16
// pairs are exact in fp32, so the result has the error of an fp32 dot product (measured against
// fp64: tests/test_gpu_stages.py::test_decoder_split_precision).  Scales keep every scaled value
// in fp16's normal range: the weights' per-matrix 2^e in the tables (DecH), the decoder inputs and
// the output gradients a power of two per wave from their largest magnitude; the hidden
// activations softplus(z) >= 0 are split unscaled (an O(1) activation below 2^-14 keeps an
// absolute error under 2^-25).  Per 64 points: forward 72 f16 MFMAs (1,152 cycles) instead of
// 192 f32 ones (6,144); backward 128 (2,048) instead of 304 (9,728).
// ---------------------------------------------------------------------------------------
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4v ldu4(const float* p) { return *reinterpret_cast<const u4v*>(p); }
__device__ __forceinline__ f4v mfma_h(u4v a, u4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}
// (ah + al)(bh + bl) without al.bl, the small terms first
__device__ __forceinline__ f4v mfma3(u4v ah, u4v al, u4v bh, u4v bl, f4v c) {
  c = mfma_h(al, bh, c);
  c = mfma_h(ah, bl, c);
  return mfma_h(ah, bh, c);
}
// two fp32 values -> their f16 hi halves and lo halves (packed pairs): hi = f16(v), lo = f16(v - hi),
// both round-to-nearest (v_cvt_pk_f16_f32; v - hi is exact in fp32).  hipcc's hazard recognizer
// does not look inside an asm string: an asm result read by an MFMA needs its wait states inside the
// string, and an asm output register must not be one a matrix-core instruction may still be reading.
// (NFI_SPLIT_ASM 1: lo halves by v_fma_mix, 4 VALU per pair instead of 5: forward 2.07 -> 2.01 ms,
//  field backward 2.02 -> 1.99 ms; 0: plain operations)
#ifndef NFI_SPLIT_ASM
#define NFI_SPLIT_ASM 1
#endif
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  const h2v h = h2v{(_Float16)a, (_Float16)b};
  hi = __builtin_bit_cast(unsigned, h);
#if NFI_SPLIT_ASM
  // lo by the mixed-precision FMA f16(hi * -1 + v), one instruction per value, in a register the
  // compiler has just written itself (the copy of hi: its own wait states cover any matrix-core
  // read still pending on that register); the string ends with the 2 wait states before an MFMA
  // reads the result
  lo = hi;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "+v"(lo) : "v"(hi), "v"(a), "v"(b));
#else
  lo = __builtin_bit_cast(unsigned, h2v{(_Float16)(a - (float)h[0]), (_Float16)(b - (float)h[1])});
#endif
}
__device__ __forceinline__ void split8(const float (&v)[8], u4v& hi, u4v& lo) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    unsigned h, o;
    split2(v[2 * w], v[2 * w + 1], h, o);
    hi[w] = h;
    lo[w] = o;
  }
}
// s = 2^e, inv = 2^-e with m s in [2^(top-1), 2^top) (e = 0 for m = 0 or not finite; |e| <= 100)
__device__ __forceinline__ void pow2_scale(float m, int top, float& s, float& inv) {
  int e = top - __builtin_amdgcn_frexp_expf(m);
  e = (m > 0.f && m < __builtin_inff()) ? min(max(e, -100), 100) : 0;
  s = __builtin_ldexpf(1.f, e);
  inv = __builtin_ldexpf(1.f, -e);
}
// softplus(z) / ln 2 (threshold z > 20) from zs = z log2(e): the ln 2 is folded into the layer-2
// table (DecH H2), one multiply fewer per hidden unit
__device__ __forceinline__ float softplus_b2(float zs) {
  const float h = __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(zs));
  return (zs > 28.8539009f) ? zs : h;
}
// the wave's 64 decoder inputs (xa/xb: channels 8q..8q+3, 8q+4..8q+7 of point 16sb + j) times a
// power of two for the wave, split; returns the inverse scale
__device__ __forceinline__ float split_inputs(const f4v xa[4], const f4v xb[4], u4v Xh[4], u4v Xl[4]) {
  float m = 0.f;
#pragma unroll
  for (int sb = 0; sb < 4; ++sb)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, fmaxf(fabsf(xa[sb][r]), fabsf(xb[sb][r])));
  float sx, isx;
  pow2_scale(wave_max_dpp(m), 15, sx, isx);
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    const float v[8] = {xa[sb][0] * sx, xa[sb][1] * sx, xa[sb][2] * sx, xa[sb][3] * sx,
                        xb[sb][0] * sx, xb[sb][1] * sx, xb[sb][2] * sx, xb[sb][3] * sx};
    split8(v, Xh[sb], Xl[sb]);
  }
  return isx;
}

// the decoder inputs of points 16sb + j (lane (j, q): channels 8q..8q+7) from the X tile, times s
__device__ __forceinline__ void split_tile_inputs(const float* __restrict__ X, int sb, float s, u4v& xh, u4v& xl) {
  const int l = lane_id(), j = l & 15, q = l >> 4;
  const f4v a = ld4(X + (16 * sb + j) * XS + 8 * q), b = ld4(X + (16 * sb + j) * XS + 8 * q + 4);
  const float v[8] = {a[0] * s, a[1] * s, a[2] * s, a[3] * s, b[0] * s, b[1] * s, b[2] * s, b[3] * s};
  split8(v, xh, xl);
}

// (NFI_FWD_XHOLD 1: the inputs split once and held across the two K-steps instead of re-read from the
//  tile and re-split per K-step: measured 2.06 vs 2.01-2.07 ms, not used)
#ifndef NFI_FWD_XHOLD
#define NFI_FWD_XHOLD 0
#endif
#ifndef NFI_FWD_PERMT
#define NFI_FWD_PERMT 1   // outputs transposed by lane swaps (1) or through the LDS tile (0)
#endif
// Decoder forward for the npts points of the wave's X tile (LDS rows of XS floats; the stale rows
// past npts are zeroed first, so they neither enter the per-wave input scale nor produce inf / NaN
// that a caller's masked sums would pick up): point l's 11 outputs.  Z^T = W1s X^T by hidden blocks hb; each K-step kb of Y^T = W2s softplus(Z)^T takes its
// B operand (hidden blocks 2kb, 2kb+1 of a point) straight from two layer-1 accumulators.  The
// inputs are re-read from the tile and split per K-step (registers: the operand tables of one
// K-step, 32, and the output accumulators, 16, stay live — the forward runs at occupancy 4).
__device__ __forceinline__ void mlp_forward_h(const float* __restrict__ dec, float* __restrict__ X, int npts,
                                              float y[NO]) {
  using H = DecH;
  const int l = lane_id(), j = l & 15, q = l >> 4;
  if (npts < 64) {   // (wave-uniform) zero the stale rows: no inf / NaN from them in the products
    if (l >= npts) {
#pragma unroll
      for (int k = 0; k < NC / 4; ++k) lds_st(reinterpret_cast<f4v*>(X + l * XS + 4 * k), f4v{0.f, 0.f, 0.f, 0.f});
    }
    wave_lds_sync();
  }
  float m = 0.f;
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    const f4v a = ld4(X + (16 * sb + j) * XS + 8 * q), b = ld4(X + (16 * sb + j) * XS + 8 * q + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, fmaxf(fabsf(a[r]), fabsf(b[r])));
  }
  float sx, isx;
  pow2_scale(wave_max_dpp(m), 15, sx, isx);
  const float cz = dec[H::SC] * isx;   // 2^-(e1 + ex) log2(e)
#if NFI_FWD_XHOLD
  u4v XH[4], XL[4];
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) split_tile_inputs(X, sb, sx, XH[sb], XL[sb]);
#endif
  f4v Y[4];
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) Y[sb] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kb = 0; kb < 2; ++kb) {
    const float* t1 = dec + H::H1 + (2 * kb * 64 + l) * 8;
    const u4v a0h = ldu4(t1), a0l = ldu4(t1 + 4), a1h = ldu4(t1 + 512), a1l = ldu4(t1 + 516);
    const f4v bz0 = ld4(dec + H::B1S + (2 * kb * 64 + l) * 4), bz1 = ld4(dec + H::B1S + ((2 * kb + 1) * 64 + l) * 4);
    const u4v a2h = ldu4(dec + H::H2 + (kb * 64 + l) * 8), a2l = ldu4(dec + H::H2 + (kb * 64 + l) * 8 + 4);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
#if NFI_FWD_XHOLD
      const u4v xh = XH[sb], xl = XL[sb];
#else
      u4v xh, xl;
      split_tile_inputs(X, sb, sx, xh, xl);
#endif
      const f4v z0 = mfma3(a0h, a0l, xh, xl, f4v{0.f, 0.f, 0.f, 0.f});
      const f4v z1 = mfma3(a1h, a1l, xh, xl, f4v{0.f, 0.f, 0.f, 0.f});
      float hv[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[r] = softplus_b2(fmaf(z0[r], cz, bz0[r]));
        hv[4 + r] = softplus_b2(fmaf(z1[r], cz, bz1[r]));
      }
      u4v hh, hl;
      split8(hv, hh, hl);
      Y[sb] = mfma3(a2h, a2l, hh, hl, Y[sb]);
    }
  }
  const float s2 = dec[H::SC + 1];
#if NFI_FWD_PERMT
  // lane (j, q) holds outputs 4q..4q+3 of point 16sb + j in Y[sb]: a 4x4 transpose of (lane row q,
  // block sb) in registers — v_permlane32_swap exchanges lanes 32-63 of its first operand with
  // lanes 0-31 of its second, v_permlane16_swap the odd 16-lane rows of the first with the even
  // rows of the second — leaves lane (j, R) with outputs 4q'..4q'+3 of point 16R + j in Y[q']
  auto swap32 = [](f4v& a, f4v& b) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[c]), __float_as_uint(b[c]), false, false);
      a[c] = __uint_as_float(r[0]);
      b[c] = __uint_as_float(r[1]);
    }
  };
  auto swap16 = [](f4v& a, f4v& b) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[c]), __float_as_uint(b[c]), false, false);
      a[c] = __uint_as_float(r[0]);
      b[c] = __uint_as_float(r[1]);
    }
  };
  swap32(Y[0], Y[2]);
  swap32(Y[1], Y[3]);
  swap16(Y[0], Y[1]);
  swap16(Y[2], Y[3]);
#pragma unroll
  for (int o = 0; o < NO; ++o) y[o] = fmaf(Y[o >> 2][o & 3], s2, dec[H::B2 + o]);
#else
  // lane (j, q) holds outputs 4q..4q+3 of point 16sb + j: transpose through the tile
  wave_lds_sync();
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    const float yv[4] = {Y[sb][0], Y[sb][1], Y[sb][2], Y[sb][3]};
    lds_store_keep(X + (16 * sb + j) * XS + 4 * q, yv);
  }
  wave_lds_sync();
#pragma unroll
  for (int o = 0; o < NO; ++o) y[o] = fmaf(X[l * XS + o], s2, dec[H::B2 + o]);
#endif
}

// Decoder input gradient for 64 points: xa/xb the decoder inputs (lane (j, q): channels 8q..8q+7
// of point 16sb + j), dY the X tile's rows (point l's 11 output gradients in columns 0..10, zeros
// in 11..15).  Calls emit(cb, sb, v) with v = dX^T (lane (j, q): channels 16cb + 4q + r of point
// 16sb + j) times post.  Two passes of two point blocks each keep the live
// registers to one K-step's tables (48), two blocks' inputs (16) and accumulators (16): the field
// backward runs at occupancy 4.
// A/B knobs of the split backward (measured, p3d_fwdbwd B=8 field backward): scheduling barriers
// between K-steps (1) / point blocks (2) 2.37-2.47 ms vs none 2.20 ms at occupancy 4 (spills) and
// 2.06 ms at occupancy 3; point blocks per pass 4 (tables loaded once) 1.89-1.90 ms vs 2 (tables
// loaded per pass) 2.06-2.07; dY operands split once and held 1.93 vs re-split per K-step 1.89-1.90.
#ifndef NFI_BWD_SB
#define NFI_BWD_SB 0
#endif
#ifndef NFI_BWD_DYHOLD
#define NFI_BWD_DYHOLD 0
#endif
#ifndef NFI_BWD_NSB
#define NFI_BWD_NSB 4   // point blocks per pass
#endif
template <class Emit>
__device__ __forceinline__ void mlp_backward_h(const float* __restrict__ dec, const f4v xa[4], const f4v xb[4],
                                               const float* __restrict__ X, float post, Emit emit) {
  using H = DecH;
  constexpr int NSB = NFI_BWD_NSB;
  const int l = lane_id(), j = l & 15, q = l >> 4;
  float m = 0.f;
#pragma unroll
  for (int sb = 0; sb < 4; ++sb)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, fmaxf(fabsf(xa[sb][r]), fabsf(xb[sb][r])));
  float sx, isx;
  pow2_scale(wave_max_dpp(m), 15, sx, isx);
  const float cz = dec[H::SC] * isx;
  // dY scale, per point (a column of every product below, so it commutes through them and comes off
  // at emit): point p's C3 max|dY_p| sy_p in [2^13, 2^14), so |d hidden| <= C3 max|dY_p sy_p| stays in
  // fp16 range.  (A per-wave scale left a point whose gradients sit 2^-20 below the wave's largest
  // with a hi / lo pair exact to 2^-2 of itself: tests/test_gpu_stages.py::test_decoder_split_wave_spread.)
  float my = 0.f;
#pragma unroll
  for (int o = 0; o < NO; ++o) my = fmaxf(my, fabsf(X[l * XS + o]));
  float syl, isyl;
  pow2_scale(my * dec[H::SC + 2], 14, syl, isyl);
  float sys[4];   // lane (j, q): the scale of point 16sb + j
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) sys[sb] = __shfl(syl, 16 * sb + j);
  const float fac = post * dec[H::SC + 3];   // 2^-(e3 + e4), times 2^-ey of the point at emit
  // 2^-e of sy = 2^e (exact)
  auto inv_pow2 = [](float v) { return __builtin_ldexpf(1.f, 1 - __builtin_amdgcn_frexp_expf(v)); };
#if NFI_BWD_DYHOLD
  // B operands of d hidden, per point block: [dY hi; dY hi] and [dY lo; dY lo] (lane (j, q): outputs
  // 8(q&1)..+7).  Against H3 = [W2 hi | W2 lo] the second adds hi.lo + lo.lo.
  u4v DH[4], DL[4];
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    const float* dr = X + (16 * sb + j) * XS + 8 * (q & 1);
    const f4v d0 = ld4(dr), d1 = ld4(dr + 4);
    const float sy = sys[sb];
    const float v[8] = {d0[0] * sy, d0[1] * sy, d0[2] * sy, d0[3] * sy, d1[0] * sy, d1[1] * sy, d1[2] * sy, d1[3] * sy};
    split8(v, DH[sb], DL[sb]);
  }
#endif
#pragma unroll
  for (int sp = 0; sp < 4 / NSB; ++sp) {
    // the second pass reloads the tables (L1 hits) instead of keeping the first pass's live: an
    // opaque zero offset keeps the compiler from merging the two passes' loads (an opaque pointer
    // would lose its global address space: flat loads)
    int zo = 0;
    asm volatile("" : "+s"(zo));
    const float* dk = dec + zo;
    u4v Xh[NSB], Xl[NSB];
#pragma unroll
    for (int s = 0; s < NSB; ++s) {
      const int sb = NSB * sp + s;
      f4v a = xa[sb], b = xb[sb];
      asm volatile("" : "+v"(a), "+v"(b));   // (split here, not hoisted into the first pass)
      const float v[8] = {a[0] * sx, a[1] * sx, a[2] * sx, a[3] * sx, b[0] * sx, b[1] * sx, b[2] * sx, b[3] * sx};
      split8(v, Xh[s], Xl[s]);
    }
    f4v gx[2][NSB];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // (no load of the next K-step's tables is hoisted above this point: they would be live
      //  beside this one's)
#if NFI_BWD_SB & 1
      __builtin_amdgcn_sched_barrier(0);
#endif
      const float* t1 = dk + H::H1 + (2 * kb * 64 + l) * 8;
      const u4v a0h = ldu4(t1), a0l = ldu4(t1 + 4), a1h = ldu4(t1 + 512), a1l = ldu4(t1 + 516);
      const f4v bz0 = ld4(dk + H::B1S + (2 * kb * 64 + l) * 4), bz1 = ld4(dk + H::B1S + ((2 * kb + 1) * 64 + l) * 4);
      const u4v a30 = ldu4(dk + H::H3 + (2 * kb * 64 + l) * 4), a31 = ldu4(dk + H::H3 + ((2 * kb + 1) * 64 + l) * 4);
      const float* t4 = dk + H::H4 + (kb * 64 + l) * 8;
      const u4v a40h = ldu4(t4), a40l = ldu4(t4 + 4), a41h = ldu4(t4 + 1024), a41l = ldu4(t4 + 1028);
#pragma unroll
      for (int s = 0; s < NSB; ++s) {
#if NFI_BWD_SB & 2
        __builtin_amdgcn_sched_barrier(0);
#endif
        const int sb = NSB * sp + s;
#if NFI_BWD_DYHOLD
        const u4v dh = DH[sb], dl = DL[sb];
#else
        // B operands of d hidden: [dY hi; dY hi] and [dY lo; dY lo] (lane (j, q): outputs
        // 8(q&1)..+7); against H3 = [W2 hi | W2 lo] the second product adds hi.lo + lo.lo
        u4v dh, dl;
        {
          const float* dr = X + (16 * sb + j) * XS + 8 * (q & 1);
          const f4v d0 = ld4(dr), d1 = ld4(dr + 4);
          const float sy = sys[sb];
          const float v[8] = {d0[0] * sy, d0[1] * sy, d0[2] * sy, d0[3] * sy,
                              d1[0] * sy, d1[1] * sy, d1[2] * sy, d1[3] * sy};
          split8(v, dh, dl);
        }
#endif
        const f4v z0 = mfma3(a0h, a0l, Xh[s], Xl[s], f4v{0.f, 0.f, 0.f, 0.f});
        const f4v z1 = mfma3(a1h, a1l, Xh[s], Xl[s], f4v{0.f, 0.f, 0.f, 0.f});
        const f4v g0 = mfma_h(a30, dh, mfma_h(a30, dl, f4v{0.f, 0.f, 0.f, 0.f}));
        const f4v g1 = mfma_h(a31, dh, mfma_h(a31, dl, f4v{0.f, 0.f, 0.f, 0.f}));
        float gv[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gv[r] = g0[r] * softplus_grad2(fmaf(z0[r], cz, bz0[r]));
          gv[4 + r] = g1[r] * softplus_grad2(fmaf(z1[r], cz, bz1[r]));
        }
        u4v gh, gl;
        split8(gv, gh, gl);
        const f4v c0 = kb ? gx[0][s] : f4v{0.f, 0.f, 0.f, 0.f}, c1 = kb ? gx[1][s] : f4v{0.f, 0.f, 0.f, 0.f};
        gx[0][s] = mfma3(a40h, a40l, gh, gl, c0);
        gx[1][s] = mfma3(a41h, a41l, gh, gl, c1);
      }
    }
#pragma unroll
    for (int s = 0; s < NSB; ++s) {
      const float f = fac * inv_pow2(sys[NSB * sp + s]);
      emit(0, NSB * sp + s, gx[0][s] * f);
      emit(1, NSB * sp + s, gx[1][s] * f);
    }
  }
}

// Dispatch: the inversion decoder on the split-f16 path, the 33-output (view-direction) decoder on
// the exact-f32 tables.  dY rows for mlp_backward: the tile's columns 0..NOUT-1, zeros up to DYC.
template <int NOUT>
constexpr int DYC = (NOUT == NO) ? 16 : 4 * DecL<NOUT>::KT;
static_assert(DYC<NOV> <= XS && DYC<NO> <= XS, "dY rows fit an X tile row");

template <int NOUT, bool PREFETCH>
__device__ __forceinline__ void mlp_forward(const float* __restrict__ dec, float* __restrict__ X, int npts,
                                            float y[NOUT]) {
  if constexpr (NOUT == NO)
    mlp_forward_h(dec, X, npts, y);
  else
    mlp_forward_tile<NOUT, PREFETCH>(dec, X, y);
}
// emit(cb, sb, v): v = dX^T block (cb, sb) (lane (j, q): channels 16cb + 4q + r of point 16sb + j)
// times post
template <int NOUT, class Emit>
__device__ __forceinline__ void mlp_backward(const float* __restrict__ dec, const f4v xa[4], const f4v xb[4],
                                             const float* __restrict__ X, float post, Emit emit) {
  if constexpr (NOUT == NO) {
    mlp_backward_h(dec, xa, xb, X, post, emit);
  } else {
    using L = DecL<NOUT>;
    const int l = lane_id(), j = l & 15, q = l >> 4;
    float gyb[4][L::KT];
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int t = 0; t < L::KT; ++t) gyb[sb][t] = X[(16 * sb + j) * XS + 4 * t + q];
    f4v gxo[2][4];
    mlp_backward_mfma<NOUT>(dec, xa, xb, gyb, gxo);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      emit(0, sb, gxo[0][sb] * post);
      emit(1, sb, gxo[1][sb] * post);
    }
  }
}

// Head: sigma = (1/alpha) * laplace_cdf(-d, beta) * (1 - mask)  (generator.py:629-636, 30-33)
//       rgb   = softmax(features) @ palette                    (generator.py:668-679)
// and the reference's other heads (nfi_field.heads, wave-uniform):
//   NFI_HEAD_NERF_DENSITY  sigma = softplus(d - 1) * (1 - mask)       (generator.py:637-641)
//   NFI_HEAD_RGB_SIGMOID   rgb = sigmoid(features[0..2]) * 2.004 - 1.002 (:665-666, :36-39);
//                          p[0..2] keeps the sigmoids for the backward
struct Head {
  float sigma;
  float rgb[3];
  float p[NA];
};

// F.softplus (beta 1, threshold 20) as ATen's CPU kernel forms it
__device__ __forceinline__ float softplus_ref(float z) { return z > 20.f ? z : log1pf(expf(z)); }

__device__ __forceinline__ void head_forward(const float y[NO], float mask, float inv_alpha, float beta,
                                             const float* __restrict__ pal, int heads, Head& h) {
  if (heads & NFI_HEAD_NERF_DENSITY) {
    h.sigma = fmul(softplus_ref(fsub(y[0], 1.f)), fsub(1.f, mask));
  } else {
    const float xn = -y[0];
    const float ex = expf(-fabsf(xn) / beta);
    const float cdf = 0.5f + 0.5f * tsign(xn) * (1.f - ex);
    h.sigma = inv_alpha * (cdf * (1.f - mask));
  }
  if (heads & NFI_HEAD_RGB_SIGMOID) {
#pragma unroll
    for (int k = 0; k < NA; ++k) h.p[k] = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float sg = 1.f / (1.f + expf(-y[1 + c]));
      h.p[c] = sg;
      h.rgb[c] = fsub(fmul(sg, 2.004f), 1.002f);
    }
    return;
  }
  float m = y[1];
#pragma unroll
  for (int k = 2; k <= NA; ++k) m = fmaxf(m, y[k]);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    h.p[k] = __expf(y[1 + k] - m);
    sum += h.p[k];
  }
  const float rs = 1.f / sum;
#pragma unroll
  for (int k = 0; k < NA; ++k) h.p[k] = h.p[k] * rs;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) a = fmaf(h.p[k], pal[k * 3 + c], a);
    h.rgb[c] = a;
  }
}

// View-direction mapper closure (generator.py:242-250, applied at :661-663) on one point: the
// colour logits are output(leaky_relu(xray + features, 0.2)) with xr the ray's mapper trunk
// output (generator.py:223-238, run.py:216-219) and vh the gain-scaled output layer ([O][32]
// weights, then [O] bias; O = 10 attention logits or 3 colour features).  y11 = {distance,
// logits zero-padded to 10} is what head_forward reads for the other fields.
__device__ __forceinline__ void viewdir_head_in(const float y[NOV], const float* __restrict__ xr,
                                                const float* __restrict__ vh, int O, float y11[NO]) {
  float hv[NVF];
#pragma unroll
  for (int k = 0; k < NVF; ++k) {
    const float pre = fadd(xr[k], y[1 + k]);
    hv[k] = pre > 0.f ? pre : fmul(pre, 0.2f);     // LeakyReLU(0.2) (ATen: x > 0 ? x : x * slope)
  }
  y11[0] = y[0];
#pragma unroll
  for (int o = 0; o < NA; ++o) {
    float acc = 0.f;
    if (o < O) {
#pragma unroll
      for (int k = 0; k < NVF; ++k) acc = fmaf(hv[k], vh[o * NVF + k], acc);
      acc = fadd(acc, vh[O * NVF + o]);
    }
    y11[1 + o] = acc;
  }
}

// Backward of viewdir_head_in: g11 = dL/d y11 -> dL/d y (33); dL/d xray = dL/d features (the sum
// xray + features passes the gradient to both).
__device__ __forceinline__ void viewdir_head_bwd(const float y[NOV], const float* __restrict__ xr,
                                                 const float* __restrict__ vh, int O, const float g11[NO],
                                                 float gy[NOV]) {
  gy[0] = g11[0];
#pragma unroll
  for (int k = 0; k < NVF; ++k) {
    float g = 0.f;
#pragma unroll
    for (int o = 0; o < NA; ++o)
      if (o < O) g = fmaf(vh[o * NVF + k], g11[1 + o], g);
    const float pre = fadd(xr[k], y[1 + k]);
    gy[1 + k] = pre > 0.f ? g : fmul(g, 0.2f);
  }
}

// ---------------------------------------------------------------------------------------
// Wave scans over per-ray arrays held as v[e] = element (e*64 + lane), chunk by chunk.
// Products and sums of the per-ray recurrences are accumulated in fp64 (ATen's CPU cumprod /
// cumsum accumulate float inputs in double).
// ---------------------------------------------------------------------------------------
// Inclusive scans on DPP (no LDS round trip): Hillis-Steele inside rows of 16 (row_shr 1, 2, 4,
// 8), then row 15's total into rows 1 and 3 and lane 31's into rows 2 and 3 (row_bcast 15 / 31).
__device__ __forceinline__ double wave_incl_prod_d(double v) {
  v *= dpp_fill<0x111>(v, 1.0);
  v *= dpp_fill<0x112>(v, 1.0);
  v *= dpp_fill<0x114>(v, 1.0);
  v *= dpp_fill<0x118>(v, 1.0);
  v *= dpp_fill<0x142, 0xA>(v, 1.0);
  v *= dpp_fill<0x143, 0xC>(v, 1.0);
  return v;
}
__device__ __forceinline__ double wave_incl_sum_d(double v) {
  v += dpp_fill<0x111>(v, 0.0);
  v += dpp_fill<0x112>(v, 0.0);
  v += dpp_fill<0x114>(v, 0.0);
  v += dpp_fill<0x118>(v, 0.0);
  v += dpp_fill<0x142, 0xA>(v, 0.0);
  v += dpp_fill<0x143, 0xC>(v, 0.0);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d);
  return v;
}

// Exclusive cumulative product T[i] = prod_{j<i} a[j]  (cumprod_exclusive, nerf_utils.py:20-25)
template <int E>
__device__ __forceinline__ void excl_prod(const float (&a)[E], float (&T)[E]) {
  double carry = 1.0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const double inc = wave_incl_prod_d((double)a[e]);
    const double ex = dpp_fill<0x138>(inc, 1.0);   // wave_shr:1, lane 0 takes 1
    T[e] = (float)(carry * ex);
    carry = carry * readlane(inc, 63);
  }
}

// ---- torch.sum of a float row on the CPU, in ATen's order ----------------------------------
// ATen's CPU sum kernel (SumKernel.cpp cascade_sum) accumulates float in FLOAT: a row of n
// contiguous values is read as n/8 vectors of 8 (the reduction kernels' Vectorized<float> width in
// this torch build), each vector lane summed by row_sum — 4 interleaved partial sums, each a
// multi_row_sum cascade of 4 levels of 16 — then the n%8 tail sequentially from 0, then the 8
// lanes in order; rows shorter than 8 take row_sum directly.  Emulated exactly (checked against
// torch 2.10 for n = 1..1023): sample_pdf's normalisation divides by this sum, and where the
// CDF's last entry rounds to 1 + 1 ulp the reference interpolates the last fine sample inside the
// last bin instead of at its end (u = 1 in deterministic mode).
__device__ __forceinline__ float aten_multi_row_sum(const float* x, int start, int step, int size) {
  // the column x[start + i*step], i < size, as multi_row_sum accumulates one of its nrows columns
  int cl2 = 0;
  while ((1 << cl2) < size) ++cl2;                           // CeilLog2
  const int lp = max(4, cl2 / 4), lstep = 1 << lp, lmask = lstep - 1;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int i = 0;
  while (i + lstep <= size) {
    for (int j = 0; j < lstep; ++j, ++i) acc[0] = fadd(acc[0], x[start + i * step]);
    for (int j = 1; j < 4; ++j) {
      acc[j] = fadd(acc[j], acc[j - 1]);
      acc[j - 1] = 0.f;
      if ((i & (lmask << (j * lp))) != 0) break;
    }
  }
  for (; i < size; ++i) acc[0] = fadd(acc[0], x[start + i * step]);
  for (int j = 1; j < 4; ++j) acc[0] = fadd(acc[0], acc[j]);
  return acc[0];
}
// row_sum over the sequence x[start + i*step], i < size (ilp factor 4)
__device__ __forceinline__ float aten_row_sum(const float* x, int start, int step, int size) {
  const int si = size / 4;
  float p[4];
  for (int k = 0; k < 4; ++k) p[k] = si ? aten_multi_row_sum(x, start + k * step, 4 * step, si) : 0.f;
  for (int i = si * 4; i < size; ++i) p[0] = fadd(p[0], x[start + i * step]);
  for (int k = 1; k < 4; ++k) p[0] = fadd(p[0], p[k]);
  return p[0];
}
// row_sum of at most 16 items with every load issued before the adds (no dependent LDS round
// trips; the multi_row_sum cascade needs >= 16 rows of 4, so none here): the same order
__device__ __forceinline__ float aten_row_sum16(const float* x, int start, int step, int size) {
  float y[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) y[i] = x[start + min(i, max(size - 1, 0)) * step];
  const int si = size / 4;
  float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i < si) p[k] = fadd(p[k], y[4 * i + k]);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i >= si * 4 && i < size) p[0] = fadd(p[0], y[i]);
  return fadd(fadd(fadd(p[0], p[1]), p[2]), p[3]);
}

// The sum of x[0..n) (wave-uniform n, x in LDS) in every lane: lanes 0..7 run the 8 vector
// lanes' row_sums side by side, lane 8 the tail, then the 8 lane results are added in order.
__device__ __forceinline__ float aten_sum_f32(const float* x, int n) {
  constexpr int VEC = 8;
  const int l = lane_id();
  float v = 0.f;
  if (n < VEC) {
    if (l == 0) v = aten_row_sum16(x, 0, 1, n);
    return readlane(v, 0);
  }
  const int V = n / VEC;
  if (l < VEC) {
    v = V <= 16 ? aten_row_sum16(x, l, VEC, V) : aten_row_sum(x, l, VEC, V);
  } else if (l == VEC) {
    float t[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) t[k] = x[min(V * VEC + k, n - 1)];
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      if (V * VEC + k < n) v = fadd(v, t[k]);
  }
  float acc = readlane(v, VEC);
#pragma unroll
  for (int k = 0; k < VEC; ++k) acc = fadd(acc, readlane(v, k));
  return acc;
}

// Ascending bitonic sort of the 64*E values v[e] (element e*64 + lane) across the wave.
template <int E>
__device__ __forceinline__ void bitonic_sort(float (&v)[E]) {
  const int l = lane_id();
  constexpr int NN = 64 * E;
#pragma unroll
  for (int k = 2; k <= NN; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int pe = e ^ (j >> 6);
          if (pe > e) {
            const bool up = ((e * 64 + l) & k) == 0;
            const float a = v[e], b = v[pe];
            v[e] = up ? fminf(a, b) : fmaxf(a, b);
            v[pe] = up ? fmaxf(a, b) : fminf(a, b);
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = e * 64 + l;
          const float o = __shfl_xor(v[e], j);
          v[e] = (((i & k) == 0) == ((i & j) == 0)) ? fminf(v[e], o) : fmaxf(v[e], o);
        }
      }
    }
  }
}

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
  R.rdn = tnorm3(R.d[0], R.d[1], R.d[2]);   // ray_directions.norm(p=2, dim=-1) (nerf_utils.py:142)
  R.near_ = a.near_[r];
  R.far_ = a.far_[r];
}

// Evaluate the field at the (up to 64) points t (one per lane; lanes >= npts ignored).
template <int NOUT, bool MLP_PREFETCH>
__device__ __forceinline__ void field_eval(const nfi_render_args& a, const PlaneView& pv, const RayCtx& R,
                                           float t, int npts, float* __restrict__ X, float& sigma,
                                           float rgb[3], int eval_base NFI_STAMP_PARAM) {
  PointP P;
  point_params(R.o, R.d, t, a.field.scene_range, pv.R, P);
  gather_features(pv, P, npts, X);
  wave_lds_sync();
  if (a.x_saved) {
    // decoder inputs for the backward: rows eval_base.. of this ray, one coalesced KiB per store
    const int N = a.fine ? 2 * a.S : a.S;
    float4* xs = reinterpret_cast<float4*>(a.x_saved + (R.r * N + eval_base) * NC);
    const int l = lane_id();
    const float* src = X + (l >> 3) * XS + 4 * (l & 7);   // row k*8 + l/8: a constant offset per k
    if (npts == 64) {
      // (the common full chunk: no per-store lane mask, so the eight LDS reads issue together
      //  instead of one exec-masked read + wait + store at a time)
#pragma unroll
      for (int k = 0; k < NC / 4; ++k) nt_store4(xs + k * 64 + l, *reinterpret_cast<const float4*>(src + k * 8 * XS));
    } else {
#pragma unroll
      for (int k = 0; k < NC / 4; ++k)
        if (8 * k + (l >> 3) < npts) nt_store4(xs + k * 64 + l, *reinterpret_cast<const float4*>(src + k * 8 * XS));
    }
  }
  NFI_STAMP(1)
  float y[NOUT];
  mlp_forward<NOUT, MLP_PREFETCH>(a.field.dec, X, npts, y);
  NFI_STAMP(2)
  if (a.y_saved && lane_id() < npts) {     // (no saved state in forward-only calls)
    const int N = a.fine ? 2 * a.S : a.S;
    float* ys = a.y_saved + R.r * NOUT * N + eval_base + lane_id();
#pragma unroll
    for (int k = 0; k < NOUT; ++k) NFI_NT_STORE(ys + k * N, y[k]);
  }
  Head h;
  if constexpr (NOUT == NOV) {
    float y11[NO];
    viewdir_head_in(y, a.field.xray + R.r * NVF, a.field.vhead, a.field.vhead_out, y11);
    head_forward(y11, P.mask, a.field.inv_alpha, a.field.beta, a.field.palette + R.b * (NA * 3), a.field.heads,
                 h);
  } else {
    head_forward(y, P.mask, a.field.inv_alpha, a.field.beta, a.field.palette + R.b * (NA * 3), a.field.heads, h);
  }
  sigma = h.sigma;
  rgb[0] = h.rgb[0];
  rgb[1] = h.rgb[1];
  rgb[2] = h.rgb[2];
  wave_lds_sync();
  NFI_STAMP(3)
}

// Ray order for L2 locality: with H, W multiples of 16 (W = a.W), physical block b (RB consecutive
// rays of one pixel row per block, RB | 16) is mapped so that the 8 XCDs (blocks are dealt
// round-robin: b and b+8 share one) each walk whole 16x16-pixel tiles, tile T going to XCD
// T % 8: the rays an XCD has in flight are a compact patch of the image, and all XCDs stay on
// nearby tiles of one image (Infinity Cache).  Bijective; identity when the shape does not tile.
__device__ __forceinline__ long long ray_of_block(unsigned b, int RB, const nfi_render_args& a) {
  const int W = a.W;
  if (W <= 0 || W % 16 || a.HW % W) return (long long)b * RB;
  const int H = a.HW / W;
  const int tx_n = W / 16, ty_n = H / 16;
  const long long tpi = (long long)tx_n * ty_n, NT = (long long)a.B * tpi;
  if (H % 16 || NT % 8) return (long long)b * RB;
  const int TBR = 16 / RB, TB = 16 * TBR;   // blocks per tile row / per tile
  const unsigned x = b & 7, k = b >> 3;
  const long long T = (long long)(k / TB) * 8 + x;
  const int j = (int)(k % TB);
  const long long img = T / tpi, rem = T % tpi;
  const int row = (int)(rem / tx_n) * 16 + j / TBR, col = (int)(rem % tx_n) * 16 + (j % TBR) * RB;
  return (img * H + row) * W + col;
}

// alpha_i = 1 - exp(-sigma_i * dist_i),  a_i = 1 - alpha_i + 1e-10  (nerf_utils.py:136-146)
__device__ __forceinline__ void alpha_of(float sigma, float dist, float& al, float& aa, float& ex) {
  ex = expf(fmul(-sigma, dist));
  al = fsub(1.f, ex);
  aa = fadd(fsub(1.f, al), 1e-10f);
}

// ---------------------------------------------------------------------------------------
// Forward kernel.  SPL = coarse samples per lane (S <= 64*SPL), NPL = merged per lane.
// ---------------------------------------------------------------------------------------
// The inversion-sized kernels (<= 128 merged samples, 11 outputs) run at occupancy 3 with the
// split-f16 decoder (168 VGPRs, 6 spilled outside the loops): 2.04 ms vs 2.57 ms at occupancy 4
// (128 VGPRs, 54 spilled).  (The exact-f32 decoder measured the other way: 2.39 at occupancy 4 vs
// 2.51 ms at 3.)
#ifndef NFI_FWD_OCC
#define NFI_FWD_OCC 3
#endif
#ifndef NFI_FWD_OCC4
#define NFI_FWD_OCC4 3   // the 256-merged-sample kernel (imagenet_256)
#endif
template <int SPL, int NPL, bool FINE, int NOUT>
__global__ void __launch_bounds__(256, (NPL <= 2 && SPL <= 2 && NOUT == NO) ? NFI_FWD_OCC
                                       : ((NPL <= 4 && SPL <= 2 && NOUT == NO) ? NFI_FWD_OCC4 : 2))
    render_fwd_kernel(nfi_render_args a) {
  constexpr bool MLP_PF = !(NOUT == NO && SPL <= 2 &&
                            ((NPL <= 2 && NFI_FWD_OCC >= 4) || (NPL <= 4 && NFI_FWD_OCC4 >= 3)));
  constexpr int SMAX = 64 * SPL, NMAX = 64 * NPL;
  // per-wave LDS: the X tile; the merge / sample_pdf arrays alias it (they are live only
  // outside field_eval), which keeps a workgroup at 36 KiB
  constexpr int WL = XTILE;
  static_assert(6 * NMAX + 2 * SMAX <= XTILE, "merge arrays must fit in the X tile");
  __shared__ __attribute__((aligned(16))) float lds[4 * WL];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = ray_of_block(blockIdx.x, 4, a) + wv;
  if (r >= nrays) return;
  NFI_STAMP_INIT
  const int S = a.S;
  const int N = FINE ? 2 * S : S;
  float* X = lds + wv * WL;
  float* Mt = X;                  // merged t     [NMAX]
  float* Ms = Mt + NMAX;          // merged sigma [NMAX]
  float* Mc = Ms + NMAX;          // merged rgb   [3][NMAX]
  int* Mi = reinterpret_cast<int*>(Mc + 3 * NMAX);   // merged -> evaluation index [NMAX]
  float* T2 = Mc + 4 * NMAX;      // [2*SMAX] coarse t | fine t (ranks); cdf | bins (sample_pdf)

  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};
  NFI_STAMP(0)

  // ---- stratified coarse depths (nerf_utils.py:104-120) ----
  float tc[SPL], sc[SPL], cc[SPL][3];
  const float delta = fdiv(fsub(R.far_, R.near_), (float)S);
#pragma unroll
  for (int e = 0; e < SPL; ++e) {
    const int i = e * 64 + l;
    float t = R.near_;
    if (i < S) {
      t = tlerp(R.near_, R.far_, fdiv((float)i, (float)S));
      if (a.randomize) {
        const float u = a.u_coarse ? a.u_coarse[r * S + i] : rng_uniform(a.seed, a.offset, r, i, 0);
        t = fadd(t, fmul(u, delta));
      }
      if (a.z_coarse) a.z_coarse[r * S + i] = t;
    }
    tc[e] = t;
    sc[e] = 0.f;
    cc[e][0] = cc[e][1] = cc[e][2] = 0.f;
    if (e * 64 < S) field_eval<NOUT, MLP_PF>(a, pv, R, t, min(64, S - e * 64), X, sc[e], cc[e], e * 64 NFI_STAMP_ARG);
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
      const float dist = (i < S - 1) ? fmul(fsub(T2[i + 1], tc[e]), R.rdn) : 0.f;
      float ex;
      alpha_of(sc[e], dist, al[e], aa[e], ex);
      if (i >= S) {
        al[e] = 0.f;
        aa[e] = 1.f;
      }
    }
    excl_prod<SPL>(aa, T);
#pragma unroll
    for (int e = 0; e < SPL; ++e) w[e] = fmul(al[e], T[e]);
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
      sm[e] = fadd(fdiv(fadd(fmaxf(wp, wi), fmaxf(wi, wn)), 2.f), 0.01f);
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < SPL; ++e) Wl[e * 64 + l] = sm[e];
    wave_lds_sync();
    // ---- sample_pdf (nerf_utils.py:185-224): bins = midpoints [S-1], weights = sm[1..S-2]
    float pw[SPL], mid[SPL];
    float* cdf = T2 + 0;        // [S-1]
    float* bins = T2 + SMAX;    // [S-1] (first the padded weights, for their sum)
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      pw[e] = (i < S - 2) ? fadd(Wl[i + 1], 1e-5f) : 0.f;
      mid[e] = (i < S - 1) ? fmul(.5f, fadd(T2[i + 1], T2[i])) : 0.f;
      if (i < S - 2) bins[i] = pw[e];
    }
    wave_lds_sync();
    // weights.sum(-1) in float, in ATen's order (the CDF's last entry, hence the bin of u = 1,
    // follows its rounding); the cumsum below accumulates in double as ATen's does
    const float totf = aten_sum_f32(bins, S - 2);
    wave_lds_sync();
    double carry = 0.0;
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      const float pdf = (i < S - 2) ? fdiv(pw[e], totf) : 0.f;
      const double inc = wave_incl_sum_d((double)pdf) + carry;
      if (i < S - 2) cdf[i + 1] = (float)inc;
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
        const int m = (lo + hi) >> 1;
        if (cdf[m] <= u) lo = m + 1;
        else hi = m;
      }
      const int below = max(0, lo - 1), above = min(S - 2, lo);
      const float c0 = cdf[below], c1 = cdf[above];
      const float b0 = bins[below], b1 = bins[above];
      float denom = fsub(c1, c0);
      denom = (denom < 1e-5f) ? 1.f : denom;
      const float tt = fdiv(fsub(u, c0), denom);
      tf[e] = fadd(b0, fmul(tt, fsub(b1, b0)));
      if (i < S && a.z_fine) a.z_fine[r * S + i] = tf[e];
      if (i >= S) tf[e] = INFINITY;
    }
    // fine depths in ascending order (each depends on its own u only, and samples at equal
    // depths have equal fields, so the order of equal values cannot change any output): the
    // merge below then needs ranks in two sorted lists instead of an O(N^2) count
    bitonic_sort<SPL>(tf);
#pragma unroll
    for (int e = 0; e < SPL; ++e)
      if (e * 64 + l >= S) tf[e] = R.near_;   // (padding back to a finite, in-box-safe depth)
    wave_lds_sync();
    NFI_STAMP(4)
    // ---- fine field evaluation (run.py:283-291) ----
    float sf[SPL], cf[SPL][3];
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      sf[e] = 0.f;
      cf[e][0] = cf[e][1] = cf[e][2] = 0.f;
      if (e * 64 < S) field_eval<NOUT, MLP_PF>(a, pv, R, tf[e], min(64, S - e * 64), X, sf[e], cf[e], S + e * 64 NFI_STAMP_ARG);
    }
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
    // stratified coarse depths are ascending up to a rounding tie-break; verify, and fall back
    // to direct counting (stable: cat order breaks ties) if not
    bool unsorted = false;
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      if (i + 1 < S) unsorted |= T2[i] > T2[i + 1];
    }
    const bool direct = __ballot(unsorted) != 0ull;
#pragma unroll
    for (int e = 0; e < SPL; ++e) {
      const int i = e * 64 + l;
      if (i < S) {
        int rc = 0, rf = 0;
        const float vc = tc[e], vf = tf[e];
        if (direct) {
          for (int j = 0; j < 2 * S; ++j) {
            const float v = T2[j];
            rc += (v < vc || (v == vc && j < i)) ? 1 : 0;
            rf += (v < vf || (v == vf && j < S + i)) ? 1 : 0;
          }
        } else {
          // coarse i: i + #fine < vc;  fine i: i + #coarse <= vf  (coarse first on ties)
          int lo = 0, hi = S;
          while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (T2[S + m] < vc) lo = m + 1;
            else hi = m;
          }
          rc = i + lo;
          lo = 0;
          hi = S;
          while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (T2[m] <= vf) lo = m + 1;
            else hi = m;
          }
          rf = i + lo;
        }
        Mt[rc] = vc;
        Ms[rc] = sc[e];
        Mi[rc] = i;
        Mt[rf] = vf;
        Ms[rf] = sf[e];
        Mi[rf] = S + i;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          Mc[k * NMAX + rc] = cc[e][k];
          Mc[k * NMAX + rf] = cf[e][k];
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
        Mi[i] = i;
#pragma unroll
        for (int k = 0; k < 3; ++k) Mc[k * NMAX + i] = cc[e][k];
      }
    }
  }
  wave_lds_sync();
  NFI_STAMP(5)

  // ---- compositing (nerf_utils.py:125-163) ----
  float t[NPL], al[NPL], aa[NPL], T[NPL];
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    const bool v = i < N;
    t[e] = v ? Mt[i] : 0.f;
    const float sg = v ? Ms[i] : 0.f;
    const float dist = (i < N - 1) ? fmul(fsub(Mt[i + 1], t[e]), R.rdn) : 0.f;
    float ex;
    alpha_of(sg, dist, al[e], aa[e], ex);
    if (!v) {
      al[e] = 0.f;
      aa[e] = 1.f;
    }
    if (v && a.t_saved) {
      a.t_saved[r * N + i] = t[e];
      a.sigma_saved[r * N + i] = sg;
#pragma unroll
      for (int k = 0; k < 3; ++k) a.rgb_saved[(r * 3 + k) * N + i] = Mc[k * NMAX + i];
      a.perm[r * N + i] = (int16_t)Mi[i];
    }
  }
  excl_prod<NPL>(aa, T);
  NFI_STAMP(6)
  if (a.tile_counts) {
    // per-tile sample counts for the backward's d-planes binning (same keys as bin_fill)
    const TileGrid Tg = tile_grid(pv.R, a.HW, a.W, N);
    const int beam = beam_of(r, a.HW, Tg);
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      const int i = e * 64 + l;
      PointP P;
      point_params(R.o, R.d, t[e], a.field.scene_range, pv.R, P);
      const bool v = i < N && P.mask == 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        int4 rec;
        const int key = plane_tile_key(P, q, beam, pv.R, Tg, r * N + i, rec);
        run_count(a.tile_counts, key, v);
      }
    }
  }
  NFI_STAMP(7)
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, sm = 0.f, sd = 0.f;
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    if (i < N) {
      const float w = fmul(al[e], T[e]);
      s0 = fmaf(w, Mc[0 * NMAX + i], s0);
      s1 = fmaf(w, Mc[1 * NMAX + i], s1);
      s2 = fmaf(w, Mc[2 * NMAX + i], s2);
      sm += w;
      sd = fmaf(w, t[e], sd);
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  sm = wave_sum(sm);
  sd = wave_sum(sd);
  if (l == 0) {
    const float bg = a.white_bg ? fsub(1.f, sm) : 0.f;
    a.rgb[r * 3 + 0] = s0 + bg;
    a.rgb[r * 3 + 1] = s1 + bg;
    a.rgb[r * 3 + 2] = s2 + bg;
    a.mask[r] = sm;
    a.depth[r] = sd;
  }
  NFI_STAMP(8)
}

// ---------------------------------------------------------------------------------------
// Backward kernel: compositing backward from saved state, then per-sample field backward
// (recompute taps + decoder), scatter-add of d planes, coordinate gradients -> d ro, d rd.
// ---------------------------------------------------------------------------------------
struct BwdArgs {
  const float* g_rgb;
  const float* g_mask;
  float* d_palette_part;  // [rays][NPL][30] per-(ray, chunk) partial dL/d palette
  float* g_ro;            // [rays][3] (NULL: no coordinate gradients)
  float* g_rd;            // [rays][3]
  float* gfeat;           // [rays][N][32] per-sample dL/d(tap feature of each plane) = dL/dx / 3
  float* gsig;            // [rays][N] dL/d sigma per merged sample
  float* wts;             // [rays][N] compositing weight per merged sample
  int npl;                // chunks of 64 per ray
  int* cursor;            // [K] tile fill cursors (NULL: bins filled by bin_fill_kernel)
  int4* list;             // [3*rays*N] tile entries
  TileGrid tg;            // tile grid of a plane
  float* d_xray;          // [rays][npl][32] per-(ray, chunk) dL/d view-direction mapper output (NFI_HEAD_VIEWDIR)
};

// One 64-sample chunk of the compositing backward's reverse scan: lane k's map x -> A_k x + B_k
// (A = a_k, B = e_k alpha_k); returns S_k = (f_{k+1} o ... o f_63)(cB), the suffix beyond lane k
// evaluated at cB (the composition of the chunks after this one at 0), and advances cB past this
// chunk.  Suffix composition on DPP: inside rows of 16 (row_shl 1, 2, 4, 8; the identity (1, 0)
// past the row's end), then each row's result composed with the totals of the rows above it (read
// from lanes 16, 32, 48 once, composed on uniform values).
__device__ __forceinline__ float suffix_affine(float A, float B, float& cB) {
  const int l = lane_id();
  {
    float A2 = dpp_fill<0x101>(A, 1.f), B2 = dpp_fill<0x101>(B, 0.f);
    B = fmaf(A, B2, B), A = A * A2;
    A2 = dpp_fill<0x102>(A, 1.f), B2 = dpp_fill<0x102>(B, 0.f);
    B = fmaf(A, B2, B), A = A * A2;
    A2 = dpp_fill<0x104>(A, 1.f), B2 = dpp_fill<0x104>(B, 0.f);
    B = fmaf(A, B2, B), A = A * A2;
    A2 = dpp_fill<0x108>(A, 1.f), B2 = dpp_fill<0x108>(B, 0.f);
    B = fmaf(A, B2, B), A = A * A2;
  }
  {
    const float a1 = readlane(A, 16), b1 = readlane(B, 16), a2 = readlane(A, 32), b2 = readlane(B, 32);
    const float a3 = readlane(A, 48), b3 = readlane(B, 48);
    const float c1a = a2 * a3, c1b = fmaf(a2, b3, b2);            // rows 2, 3
    const float c0a = a1 * c1a, c0b = fmaf(a1, c1b, b1);          // rows 1, 2, 3
    const int row = l >> 4;
    const float ca = row == 0 ? c0a : (row == 1 ? c1a : (row == 2 ? a3 : 1.f));
    const float cb = row == 0 ? c0b : (row == 1 ? c1b : (row == 2 ? b3 : 0.f));
    B = fmaf(A, cb, B);
    A = A * ca;
  }
  const float An = dpp_fill<0x130>(A, 1.f), Bn = dpp_fill<0x130>(B, 0.f);   // wave_shl:1
  const float Sk = fmaf(An, cB, Bn);                       // lane 63: the identity -> cB
  cB = fmaf(readlane(A, 0), cB, readlane(B, 0));
  return Sk;
}

// Compositing backward (nerf_utils.py:125-163 under autograd), one wave per ray:
// dL/d alpha_k = T_k (e_k - S_k), S_k = sum_{i>k} e_i alpha_i prod_{k<j<i} a_j (reverse affine
// scan), e_i = g_rgb.c_i + g_mask(-white bg) -> dL/d sigma_i, weights w_i, and the ||rd|| term.
template <int NPL>
__global__ void __launch_bounds__(256) composite_bwd_kernel(nfi_render_args a, BwdArgs g) {
  constexpr int NMAX = 64 * NPL;
  __shared__ float lds[4 * (NMAX + 8)];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = ray_of_block(blockIdx.x, 4, a) + wv;
  if (r >= nrays) return;
  const int N = a.fine ? 2 * a.S : a.S;
  float* Lt = lds + wv * (NMAX + 8);
  RayCtx R;
  load_ray(a, r, R);
  const float gr0 = g.g_rgb[r * 3 + 0], gr1 = g.g_rgb[r * 3 + 1], gr2 = g.g_rgb[r * 3 + 2];
  const float gm = g.g_mask[r] - (a.white_bg ? (gr0 + gr1 + gr2) : 0.f);
  float t[NPL], sg[NPL], al[NPL], aa[NPL], ex[NPL], dist[NPL], raw[NPL], T[NPL], ee[NPL];
  float c0[NPL], c1[NPL], c2[NPL];
  // every load issues up front at a clamped index (a branch around a load makes the compiler
  // wait for it before the next one); the lanes past N take their zeros by selects below
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int ic = min(e * 64 + l, N - 1);
    t[e] = a.t_saved[r * N + ic];
    sg[e] = a.sigma_saved[r * N + ic];
    c0[e] = a.rgb_saved[(r * 3 + 0) * N + ic];
    c1[e] = a.rgb_saved[(r * 3 + 1) * N + ic];
    c2[e] = a.rgb_saved[(r * 3 + 2) * N + ic];
  }
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    t[e] = (e * 64 + l < N) ? t[e] : 0.f;
    Lt[e * 64 + l] = t[e];
  }
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int i = e * 64 + l;
    const bool v = i < N;
    sg[e] = v ? sg[e] : 0.f;
    raw[e] = (i < N - 1) ? fsub(Lt[min(i + 1, NMAX - 1)], t[e]) : 0.f;
    dist[e] = fmul(raw[e], R.rdn);
    alpha_of(sg[e], dist[e], al[e], aa[e], ex[e]);
    al[e] = v ? al[e] : 0.f;
    aa[e] = v ? aa[e] : 1.f;
    ee[e] = v ? (gr0 * c0[e] + gr1 * c1[e] + gr2 * c2[e]) + gm : 0.f;
  }
  excl_prod<NPL>(aa, T);
  float grdn = 0.f;
  float cB = 0.f;   // composition of the maps beyond the current chunk, evaluated at 0
#pragma unroll
  for (int e = NPL - 1; e >= 0; --e) {
    const int i = e * 64 + l;
    // suffix composition of the maps x -> A x + B on DPP: inside rows of 16 (row_shl 1, 2, 4, 8;
    // the identity (1, 0) past the row's end), then each row's result composed with the totals of
    // the rows above it (read from lanes 16, 32, 48 once, composed on uniform values)
    const float Sk = suffix_affine(aa[e], ee[e] * al[e], cB);
    const float dal = T[e] * (ee[e] - Sk);                   // dL/d alpha_k
    grdn += dal * sg[e] * ex[e] * raw[e];                    // dists = raw * ||rd||
    if (i < N) {
      g.gsig[r * N + i] = dal * dist[e] * ex[e];             // d alpha/d sigma = dist * exp(-sigma dist)
      g.wts[r * N + i] = al[e] * T[e];                       // w_i; dL/d c_i = w_i g_rgb
    }
  }
  if (g.g_ro) {
    grdn = wave_sum(grdn);
    if (l < 3) {
      g.g_ro[r * 3 + l] = 0.f;
      // (R.d by a select, not R.d[l]: a lane-indexed RayCtx is a memory object the compiler puts in LDS)
      const float dl = l == 0 ? R.d[0] : (l == 1 ? R.d[1] : R.d[2]);
      g.g_rd[r * 3 + l] = grdn * (dl / R.rdn);               // d rd += d||rd|| * rd / ||rd||
    }
  }
}

// Field backward for one chunk of 64 merged samples of one ray (one wave): recompute taps
// and decoder, sigma/colour head backward, decoder input-gradient, per-sample feature
// gradient -> gfeat (d planes is summed per tile afterwards), palette partial, and the
// grid_sampler_2d d-grid -> d ray origins/directions (re-gather, generator.py:312-326).
// (occupancy 3: the split decoder backward holds its 48 table registers, the four point blocks'
//  inputs and accumulators at 162 VGPRs without spills: 1.89 ms vs 2.20 ms at occupancy 4 with spills)
#ifndef NFI_FIELD_OCC
#define NFI_FIELD_OCC 3
#endif
#ifndef NFI_BIN_BATCH
#define NFI_BIN_BATCH 1
#endif
// VARIANT = false: the inversion field (heads == 0 at compile time, the register budget of the
// hot path is not shared with the other heads); true: nfi_field.heads read at run time.
// NOUT = 33: the view-direction mapper field (NFI_HEAD_VIEWDIR, always with VARIANT).
template <bool VARIANT, int NOUT>
__global__ void __launch_bounds__(256, NOUT == NO ? NFI_FIELD_OCC : 2) field_bwd_kernel(nfi_render_args a, BwdArgs g) {
  __shared__ __attribute__((aligned(16))) float lds[4 * XTILE];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  // (npl chunks per ray, 4 jobs per block: 4 / npl rays per block)
  const long long job = (g.npl <= 4 && 4 % g.npl == 0)
                            ? ray_of_block(blockIdx.x, 4 / g.npl, a) * g.npl + wv
                            : (long long)blockIdx.x * 4 + wv;
  const long long r = job / g.npl;
  const int e = (int)(job % g.npl);
  if (r >= nrays) return;
  const int N = a.fine ? 2 * a.S : a.S;
  if (e * 64 >= N) return;
  NFI_STAMP_INIT
  float* X = lds + wv * XTILE;
  const float sr = a.field.scene_range;
  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};
  const float* pal = a.field.palette + R.b * (NA * 3);
  const float gr0 = g.g_rgb[r * 3 + 0], gr1 = g.g_rgb[r * 3 + 1], gr2 = g.g_rgb[r * 3 + 2];
  NFI_STAMP(16)

  const int i = e * 64 + l;
  const bool v = i < N;
  // every per-sample load is issued at a clamped valid index and masked by a select afterwards
  // (a lane-guarded load becomes an exec-mask branch with a vmcnt(0) wait after it)
  const long long ic = r * N + min(i, N - 1);
  const float t_ld = a.t_saved[ic];
  const int p_ld = (int)a.perm[ic];
  const float gs_ld = g.gsig[ic], w_ld = g.wts[ic];
  const float te = v ? t_ld : R.near_;
  const int ei = v ? p_ld : 0;
  float pmask;
  {
    PointP P;
    point_params(R.o, R.d, te, sr, pv.R, P);
    pmask = P.mask;
  }
  // decoder inputs saved by the forward (no re-gather here), loaded straight into the MFMA
  // operand layout: lane (j, q) takes channels 8q..8q+7 of points 16sb + j
  // (point 16sb + j's evaluation index is lane 16sb + j's ei: one ds_bpermute each instead of a
  //  dependent perm load per block, so the 8 row loads issue together)
  f4v xa[4], xb[4];
  {
    const int j = l & 15, q = l >> 4;
    int eis[4];
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) eis[sb] = __shfl(ei, 16 * sb + j);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      // (points past N have ei = 0: row 0 of this ray is loaded and zeroed by the select)
      const float* xr = a.x_saved + (r * N + eis[sb]) * NC + 8 * q;
      xa[sb] = ld4(xr);
      xb[sb] = ld4(xr + 4);
    }
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const bool vp = e * 64 + 16 * sb + j < N;
      const f4v z{0.f, 0.f, 0.f, 0.f};
      xa[sb] = vp ? xa[sb] : z;
      xb[sb] = vp ? xb[sb] : z;
    }
  }
  NFI_STAMP(17)
  // decoder outputs saved by the forward (no forward MLP here)
  float y[NOUT];
  {
    const float* ys = a.y_saved + r * NOUT * N + ei;
#pragma unroll
    for (int k = 0; k < NOUT; ++k) y[k] = ys[k * N];
#pragma unroll
    for (int k = 0; k < NOUT; ++k) y[k] = v ? y[k] : 0.f;
  }
  float gy[NO];
  float y11[NO];
  if constexpr (NOUT == NOV) {
    viewdir_head_in(y, a.field.xray + r * NVF, a.field.vhead, a.field.vhead_out, y11);
  } else {
#pragma unroll
    for (int k = 0; k < NO; ++k) y11[k] = y[k];
  }
  {
    Head h;
    const int heads = VARIANT ? a.field.heads : 0;
    head_forward(y11, pmask, a.field.inv_alpha, a.field.beta, pal, heads, h);
    const float gs = v ? gs_ld : 0.f;
    if (heads & NFI_HEAD_NERF_DENSITY) {
      // sigma -> d: softplus_backward of d - 1 (ATen: z > 20 ? g : g * e^z / (e^z + 1)), :637-641
      const float z = fsub(y11[0], 1.f);
      const float gm = fmul(gs, fsub(1.f, pmask));
      const float ez = expf(z);
      gy[0] = z > 20.f ? gm : gm * (ez / (ez + 1.f));
    } else {
      // sigma -> distance  (generator.py:629-636, laplace_cdf generator.py:30-33)
      const float xn = -y11[0];
      const float sgn = tsign(xn);
      const float ex2 = expf(-fabsf(xn) / a.field.beta);
      const float gcdf = (gs * a.field.inv_alpha) * (1.f - pmask);
      gy[0] = -(((gcdf * 0.5f * sgn) * ex2 / a.field.beta) * sgn);
    }
    const float w = v ? w_ld : 0.f;
    const float gc0 = w * gr0, gc1 = w * gr1, gc2 = w * gr2;
    if (heads & NFI_HEAD_RGB_SIGMOID) {
      // rgb -> features: (g * 2.004) * (1 - s) * s  (sigmoid backward), no palette
      const float gc[3] = {gc0, gc1, gc2};
#pragma unroll
      for (int k = 0; k < NA; ++k) gy[1 + k] = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c) gy[1 + c] = fmul(fmul(gc[c], 2.004f), fsub(1.f, h.p[c])) * h.p[c];
    } else {
      // rgb -> logits (softmax backward) and palette gradient  (generator.py:668-679)
      float gp[NA], dot = 0.f;
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        gp[k] = gc0 * pal[k * 3 + 0] + gc1 * pal[k * 3 + 1] + gc2 * pal[k * 3 + 2];
        dot = fmaf(gp[k], h.p[k], dot);
      }
#pragma unroll
      for (int k = 0; k < NA; ++k) gy[1 + k] = (gp[k] - dot) * h.p[k];
      // the chunk's palette partial sum_i p_k(i) gc_c(i) = g_rgb_c(ray) sum_i w_i p_k(i) (the
      // upstream rgb gradient is one per ray): ten wave sums on DPP (fixed order), no LDS
      float pw[NA];
#pragma unroll
      for (int k = 0; k < NA; ++k) pw[k] = wave_sum(h.p[k] * w);
      const int lk = l / 3, lc = l - 3 * lk;
      float sel = pw[0];
#pragma unroll
      for (int k = 1; k < NA; ++k) sel = (lk == k) ? pw[k] : sel;
      const float grc = (lc == 0) ? gr0 : ((lc == 1) ? gr1 : gr2);
      if (l < NA * 3) g.d_palette_part[(r * g.npl + e) * (NA * 3) + l] = sel * grc;
    }
  }
  // dY^T operands through the tile: row = point, 4 KT columns (NOUT outputs + zeros)
  float gyo[NOUT];
  if constexpr (NOUT == NOV) {
    viewdir_head_bwd(y, a.field.xray + r * NVF, a.field.vhead, a.field.vhead_out, gy, gyo);
  } else {
#pragma unroll
    for (int k = 0; k < NO; ++k) gyo[k] = gy[k];
  }
  wave_lds_sync();
  {
    float dyr[DYC<NOUT>];
#pragma unroll
    for (int o = 0; o < DYC<NOUT>; ++o) dyr[o] = (o < NOUT) ? gyo[o] : 0.f;
    lds_store_keep(X + l * XS, dyr);
  }
  wave_lds_sync();
  if constexpr (NOUT == NOV) {
    // dL/d xray of this ray chunk: column sums of the feature gradients (tile columns 1..32)
    const int col = l & 31, r0 = (l >> 5) * 32;
    float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) s4[jj & 3] += X[(r0 + jj) * XS + 1 + col];
    const float sh = sum_halves((s4[0] + s4[1]) + (s4[2] + s4[3]));
    // per-(ray, chunk) partial, summed over the chunks by the caller in a fixed order (no float
    // atomics: the mapper's gradients are bitwise reproducible)
    if (l < NVF) g.d_xray[(r * g.npl + e) * NVF + l] = sh;
  }
  NFI_STAMP(18)
  // x = (e1+e2+e3)/3: each plane's tap feature gradient is dX/3.  Lane (j, q) holds channels
  // 16cb + 4q.. of point 16sb + j
  {
    const int j = l & 15, q = l >> 4;
    float* gf = g.gfeat + (r * N + e * 64 + j) * NC + 4 * q;
    mlp_backward<NOUT>(a.field.dec, xa, xb, X, 1.f / 3.f, [&](int cb, int sb, f4v gv) {
      if (e * 64 + 16 * sb + j < N) *reinterpret_cast<f4v*>(gf + 16 * sb * NC + 16 * cb) = gv;
    });
  }
  NFI_STAMP(19)
  NFI_STAMP(20)
  if (g.cursor) {
    // append this sample's three (plane, tile) entries to the d-planes bins
    PointP P;
    point_params(R.o, R.d, te, sr, pv.R, P);
    const bool vb = v && P.mask == 0.f;
    const int beam = beam_of(r, a.HW, g.tg);
#if NFI_BIN_BATCH
    // the three cursor atomics issued together (one return latency instead of three in a row),
    // then the three record stores
    int4 rec[3];
    int key[3], old[3];
    LaneRuns lr[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      key[q] = plane_tile_key(P, q, beam, pv.R, g.tg, r * N + i, rec[q]);
      lr[q] = lane_runs(key[q], vb);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      old[q] = 0;
      if (lr[q].start && vb) old[q] = atomicAdd(g.cursor + key[q], lr[q].len);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int pos = __shfl(old[q], lr[q].leader) + (lane_id() - lr[q].leader);
      if (vb) g.list[pos] = rec[q];
    }
#else
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      int4 rec;
      const int key = plane_tile_key(P, q, beam, pv.R, g.tg, r * N + i, rec);
      const int pos = run_increment(g.cursor, key, vb);
      if (vb) g.list[pos] = rec;
    }
#endif
  }
  NFI_STAMP(21)
}

struct BinArgs {
  const float* ro;
  const float* rd;
  const float* t;        // [rays][N] merged depths (saved by the forward)
  long long nsamp;       // rays * N
  int N, HW, R;
  TileGrid tg;
  float sr;
  int* counts;           // [K]
  int* cursor;           // [K]
  int4* list;            // [3 * nsamp] entries {sample, local cell key, w bits, n bits}
};

// Tile keys of sample s for the three planes, and each plane's entry record {s, local cell key,
// w, n} (key = ly << 16 | lx << 8 | ox | oy << 1 inside the tile); false for samples outside
// the box (their gradient is exactly zero: sigma * (1 - mask) and weight 0).
__device__ __forceinline__ bool sample_keys(const BinArgs& A, long long s, int key[3], int4 rec[3]) {
  const long long ray = s / A.N;
  const int beam = beam_of(ray, A.HW, A.tg);
  float o[3], d[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    o[k] = A.ro[ray * 3 + k];
    d[k] = A.rd[ray * 3 + k];
  }
  PointP P;
  point_params(o, d, A.t[s], A.sr, A.R, P);
#pragma unroll
  for (int q = 0; q < 3; ++q) key[q] = plane_tile_key(P, q, beam, A.R, A.tg, s, rec[q]);
  return P.mask == 0.f;
}

__global__ void __launch_bounds__(256) bin_count_kernel(BinArgs A) {
  const long long s = (long long)blockIdx.x * 256 + threadIdx.x;
  int key[3] = {0, 0, 0};
  int4 rec[3];
  bool v = s < A.nsamp;
  if (v) v = sample_keys(A, s, key, rec);
#pragma unroll
  for (int q = 0; q < 3; ++q) run_count(A.counts, key[q], v);
}

__global__ void __launch_bounds__(256) bin_fill_kernel(BinArgs A) {
  const long long s = (long long)blockIdx.x * 256 + threadIdx.x;
  int key[3] = {0, 0, 0};
  int4 rec[3];
  bool v = s < A.nsamp;
  if (v) v = sample_keys(A, s, key, rec);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int pos = run_increment(A.cursor, key[q], v);
    if (v) A.list[pos] = rec[q];
  }
}

// Exclusive scans over the K tile counts: offsets (entry starts; cursor := offsets) and
// chunk starts (ceil(count / CHUNK) workgroup chunks per tile); total chunks -> meta[0].
// Two passes over 1024-tile blocks: block partial sums, then each block scans its tiles after
// summing the partials of the blocks before it (K/1024 of them).
__device__ __forceinline__ int wave_incl_scan_i(int v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(v, d);
    if (l >= d) v += t;
  }
  return v;
}

// inclusive block scan of (a, b) pairs over 1024 threads; returns block totals via tot
__device__ __forceinline__ void block_scan2(int& a, int& b, int& ta, int& tb) {
  __shared__ int sa[16], sbx[16];
  const int wv = threadIdx.x >> 6, l = lane_id();
  a = wave_incl_scan_i(a);
  b = wave_incl_scan_i(b);
  if (l == 63) {
    lds_st(sa + wv, a);
    lds_st(sbx + wv, b);
  }
  __syncthreads();
  int pa = 0, pb = 0;
  ta = 0;
  tb = 0;
  for (int k = 0; k < 16; ++k) {
    if (k < wv) {
      pa += sa[k];
      pb += sbx[k];
    }
    ta += sa[k];
    tb += sbx[k];
  }
  a += pa;
  b += pb;
  __syncthreads();
}

__global__ void __launch_bounds__(1024) scan_partials_kernel(const int* __restrict__ counts, int K,
                                                             int* __restrict__ part) {
  const int k = blockIdx.x * 1024 + threadIdx.x;
  const int c = (k < K) ? counts[k] : 0;
  int a = c, b = (c + CHUNK - 1) / CHUNK, ta, tb;
  block_scan2(a, b, ta, tb);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ta;
    part[2 * blockIdx.x + 1] = tb;
  }
}

__global__ void __launch_bounds__(1024) scan_blocks_kernel(const int* __restrict__ counts, int K,
                                                           const int* __restrict__ part,
                                                           int* __restrict__ offsets, int* __restrict__ cursor,
                                                           int* __restrict__ chunk_start, int* __restrict__ meta) {
  // prefix of the blocks before this one
  int pa = 0, pb = 0;
  for (int q = threadIdx.x; q < (int)blockIdx.x; q += 1024) {
    pa += part[2 * q];
    pb += part[2 * q + 1];
  }
  int ta, tb;
  block_scan2(pa, pb, ta, tb);   // (only the totals are used)
  const int k = blockIdx.x * 1024 + threadIdx.x;
  const int c = (k < K) ? counts[k] : 0;
  const int cc = (c + CHUNK - 1) / CHUNK;
  int a = c, b = cc, ua, ub;
  block_scan2(a, b, ua, ub);
  if (k < K) {
    offsets[k] = ta + a - c;
    cursor[k] = ta + a - c;
    chunk_start[k] = tb + b - cc;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 1023) {
    offsets[K] = ta + a;
    chunk_start[K] = tb + b;
    meta[0] = tb + b;
  }
}

// chunk -> tile map (one dependent load per chunk in tile_accum instead of a binary search); block
// 0 also zeroes the 64 list records after the last entry, which the tile pass's record prefetch
// reads past the end (a zero record: slot 0, weights 0)
__global__ void __launch_bounds__(256) chunk_map_kernel(const int* __restrict__ counts,
                                                        const int* __restrict__ chunk_start, int K,
                                                        int* __restrict__ chunk_tile,
                                                        const int* __restrict__ offsets, int4* __restrict__ list) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 64) list[offsets[K] + threadIdx.x] = make_int4(0, 0, 0, 0);
  if (k >= K) return;
  const int c0 = chunk_start[k], nc = (counts[k] + CHUNK - 1) / CHUNK;
  for (int j = 0; j < nc; ++j) chunk_tile[c0 + j] = k;
}

// ---- deterministic mode (nfi_set_deterministic): the entries of every tile ordered by sample
// index (their append order otherwise follows the cursor atomics), and the d planes summed from the
// chunks' partial tile images in a fixed order (no float atomics): a backward whose results are
// bitwise reproducible run to run.
// One workgroup per chunk (the tile pass's chunks: <= CHUNK entries of one tile): each of its
// entries' rank = the number of the tile's entries with a smaller sample index (unique within a
// tile: one entry per sample and plane), counted against the tile's keys staged through LDS 1,024
// at a time; the entry is copied to its rank.  O(CHUNK n / 256) per chunk of an n-entry tile — a
// reproducibility mode, not the product path.
constexpr int DET_PER = CHUNK / 256;
static_assert(CHUNK % 256 == 0 && CHUNK >= 256, "det_sort_kernel ranks CHUNK / 256 entries per thread");
__global__ void __launch_bounds__(256) det_sort_kernel(const int4* __restrict__ list, const int* __restrict__ offsets,
                                                       const int* __restrict__ chunk_start,
                                                       const int* __restrict__ chunk_tile, const int* __restrict__ meta,
                                                       int4* __restrict__ sorted) {
  const int c = blockIdx.x;
  if (c >= meta[0]) return;
  const int tile = chunk_tile[c];
  const int a = offsets[tile], n = offsets[tile + 1] - a;
  const int first = (c - chunk_start[tile]) * CHUNK, last = min(n, first + CHUNK);
  __shared__ int ks[1024];
  const int tid = threadIdx.x;
  int my[DET_PER], rank[DET_PER];
#pragma unroll
  for (int j = 0; j < DET_PER; ++j) {
    const int e = first + tid + 256 * j;
    my[j] = e < last ? list[a + e].x : 0x7fffffff;
    rank[j] = 0;
  }
  for (int j0 = 0; j0 < n; j0 += 1024) {
    const int m = min(1024, n - j0);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 256 * j;
      if (t < m) ks[t] = list[a + j0 + t].x;
    }
    __syncthreads();
    for (int t = 0; t < m; ++t) {
      const int v = ks[t];
#pragma unroll
      for (int j = 0; j < DET_PER; ++j) rank[j] += v < my[j] ? 1 : 0;
    }
  }
#pragma unroll
  for (int j = 0; j < DET_PER; ++j) {
    const int e = first + tid + 256 * j;
    if (e < last) sorted[a + rank[j]] = list[a + e];
  }
}
// the 64 zeroed records after the last entry that the tile pass's record prefetch reads
__global__ void det_pad_kernel(const int* __restrict__ offsets, int K, int4* __restrict__ sorted) {
  sorted[offsets[K] + threadIdx.x] = make_int4(0, 0, 0, 0);
}
// d planes += the partial tile images [chunk][TTX*TTY][NC] of every tile covering the texel: tiles
// by (beam, ty, tx) ascending, each tile's chunks ascending.  One thread per (b, q, y, x, channel).
__global__ void __launch_bounds__(256) dplanes_reduce_kernel(const float* __restrict__ part,
                                                             const int* __restrict__ chunk_start, TileGrid G, int B,
                                                             int R, long long sb, int sq, int st,
                                                             float* __restrict__ dplanes) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)B * 3 * R * R * NC) return;
  const int ch = (int)(i % NC);
  long long t = i / NC;
  const int x = (int)(t % R);
  t /= R;
  const int y = (int)(t % R);
  t /= R;
  const int q = (int)(t % 3), b = (int)(t / 3);
  // tiles whose 8 x 5 texels hold (x, y): x - TSX tx in [0, TSX], y - TSY ty in [0, TSY]
  const int tx0 = max(0, (x - TSX + TSX - 1) / TSX), tx1 = min(G.nx - 1, x / TSX);
  const int ty0 = max(0, (y - TSY + TSY - 1) / TSY), ty1 = min(G.ny - 1, y / TSY);
  float v = 0.f;
  const int nb = beams_per_image(G);
  for (int bm = 0; bm < nb; ++bm)
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) {
        const int key = tile_key(b * nb + bm, q, tx, ty, G);
        const int slot = ((y - TSY * ty) * TTX + (x - TSX * tx)) * NC + ch;
        for (int c = chunk_start[key]; c < chunk_start[key + 1]; ++c) v += part[(long long)c * (TTX * TTY * NC) + slot];
      }
  if (v != 0.f) dplanes[(long long)b * sb + (long long)q * sq + (long long)(y * R + x) * st + ch] += v;
}

struct TileArgs {
  const float* planes;    // texel-major, strides sb / sq / st as dplanes
  float* dpc;             // grid gradients, dpc_at() layout (NULL: no pose gradients)
  const float* gfeat;     // [nsamp][32]
  const int* counts;
  const int* offsets;
  const int* chunk_start; // [K+1]
  const int* chunk_tile;  // [total chunks]
  int* meta;              // meta[0] = total chunks, meta[1] = the tile pass's chunk queue
  const int4* list;
  float* dplanes;
  long long sb;
  int sq, st;
  int R;
  TileGrid tg;
  // integrity checks of the -DNFI_TILE_CHECK debug build (unused by the product kernels)
  const int* cursor;      // [K] bin cursors after the append: must equal offsets + counts
  int* check;             // [64] violation counters / first-failure record (tile_fail)
  float* shadow;          // d planes summed a second way (per-entry float atomics), same strides
  long long nsamp;
  int K;
  // deterministic mode (nfi_set_deterministic): each chunk's merged tile image [TTX*TTY][NC] is
  // stored here instead of flushed with float atomics; dplanes_reduce_kernel sums them in order
  float* part;
};

typedef float img32 __attribute__((ext_vector_type(32)));

// ---- -DNFI_TILE_CHECK: device-side integrity checks of the tile pass ----
// Every global index the pass derives from loaded or shuffled data, every LDS region it stages
// and reads back, and the bin lists themselves are checked; a violation increments
// check[code] and records the first failure (code, chunk, tile, lane, value, expected) in
// check[32..37] instead of trapping, and the index is clamped so the launch still completes (a
// faulting kernel would take the GPU down).  The host reads the counters after the launch and
// fails the call with NFI_ECHECK.  Codes:
//   1 chunk / tile / entry range      2 bin list incomplete (cursor != offsets + counts)
//   3 record sample index >= nsamp    4 record slot > 30 or unknown flag bits
//   5 shuffled row index != record    6 scalar entry record != vector record
//   7 gradient-row stage read back    8 tile texels read back after staging
//   9 wave-image dump read back      10 record weights not in [0, 1]
//  11 tile texels changed during the chunk   12 gradient-row stage changed during the entry loop
#ifndef NFI_TILE_CHECK
#define NFI_TILE_CHECK 0
#endif
#if NFI_TILE_CHECK
__device__ __noinline__ void tile_fail(int* check, int code, int c, int tile, int lane, long long v,
                                       long long expect) {
  atomicAdd(check + code, 1);
  if (atomicCAS(check + 31, 0, code) == 0) {
    check[32] = code;
    check[33] = c;
    check[34] = tile;
    check[35] = lane;
    check[36] = (int)v;
    check[37] = (int)expect;
  }
}
#define NFI_TCHK(cond, code, c, tile, lane, v, e) \
  if (!(cond)) tile_fail(A.check, code, c, tile, lane, (long long)(v), (long long)(e))
#endif
typedef int iv4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) iv4* cint4_p;

// gradient-row stage: BATCH rows of XS = 36 floats per wave (the 4-float pad makes both the
// per-lane b128 row stores / reads and the per-entry row reads conflict-free, with
// immediate-offset addressing).  60 rows, not 64, so that the stages, the tile texels and 4
// workgroups fit one CU's LDS; the stage (2,160 floats) still holds a wave's 2,048-float image.
#ifndef NFI_TILE_BATCH
#define NFI_TILE_BATCH 56
#endif
constexpr int BATCH = NFI_TILE_BATCH;
constexpr int TROWS = BATCH * XS;   // floats per wave
__device__ __forceinline__ int stage_at(int u, int c) { return u * XS + c; }
__device__ __forceinline__ int stage_q(int u, int k) { return u * XS + 4 * k; }
// the tile's 8x5 plane texels x 32 channels (pose gradients), texel rows of XS floats (per-lane
// b128 reads of different texels conflict only for texels 16 slots apart); a tile row of 8
// texels is TEXR floats
constexpr int TEXR = TTX * XS;
constexpr int TEXF = TTY * TEXR;                // 1,440 floats
__device__ __forceinline__ int tex_at(int texel) { return (texel / TTX) * TEXR + (texel % TTX) * XS; }
// (the wave images are dumped over the stages and texels at the end of a chunk: >= 4 x 2,048)
constexpr int TILE_LDS = (4 * TROWS + TEXF > 4 * 2048) ? 4 * TROWS + TEXF : 4 * 2048;   // 38,016 B at BATCH 56

// One entry into the register image: img[slot] += gw (1 - w), img[slot + 1] += gw w, for a
// wave-uniform slot (0..30), through a wave-uniform JUMP TABLE — 31 static cases, one per slot, each
// two VOP2 v_fmac_f32 on fixed registers of the image (pinned to v[40:71] so the cases can name them),
// a branch to the common exit and padding to 16 B.  The case address is PC-relative: s_getpc_b64 +
// slot * 16 + the table's offset (an assembler-resolved label difference, s_lshl4_add_u32), then
// s_setpc_b64.  No GPR-index mode (s_set_gpr_idx_on) and no M0: register writes returning from loads
// in flight are never redirected (round 5 measured that hazard class under index mode).
// Per entry: gw, 1 - w and the case's two FMAs (5 VALU) plus one table jump, whatever the cell
// sequence; scripts/isa_lint.py rule 6 checks every table of the build against its slot registers.
// (y-weights: half 0 of the wave holds texel row ly with weight 1 - n, half 1 row ly + 1 with n.)
__device__ __forceinline__ void tile_entry(img32& img, int slot, float w, float nn, float g, float wsgn,
                                           float woff) {
  const float gw = g * fmaf(nn, wsgn, woff);
  const float omw = 1.f - w;
  slot = min((unsigned)slot, 30u);   // (cells are slots 0..30; never leave the table, whatever the record)
#define NFI_JF(D0, D1) "v_fmac_f32 v" #D0 ", %2, %3\n\tv_fmac_f32 v" #D1 ", %4, %2\n\ts_branch 3f\n\ts_nop 0\n\t"
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "1:\n\t"
      "s_lshl4_add_u32 s90, %1, 2f-1b\n\t"
      "s_add_u32 s88, s88, s90\n\t"
      "s_addc_u32 s89, s89, 0\n\t"
      "s_setpc_b64 s[88:89]\n"
      "2:\n\t"
      NFI_JF(40, 41) NFI_JF(41, 42) NFI_JF(42, 43) NFI_JF(43, 44) NFI_JF(44, 45) NFI_JF(45, 46)
      NFI_JF(46, 47) NFI_JF(47, 48) NFI_JF(48, 49) NFI_JF(49, 50) NFI_JF(50, 51) NFI_JF(51, 52)
      NFI_JF(52, 53) NFI_JF(53, 54) NFI_JF(54, 55) NFI_JF(55, 56) NFI_JF(56, 57) NFI_JF(57, 58)
      NFI_JF(58, 59) NFI_JF(59, 60) NFI_JF(60, 61) NFI_JF(61, 62) NFI_JF(62, 63) NFI_JF(63, 64)
      NFI_JF(64, 65) NFI_JF(65, 66) NFI_JF(66, 67) NFI_JF(67, 68) NFI_JF(68, 69) NFI_JF(69, 70)
      NFI_JF(70, 71)
      "3:"
      : "+{v[40:71]}"(img)
      : "s"(slot), "v"(gw), "v"(omw), "s"(w)
      : "s88", "s89", "s90", "scc");
#undef NFI_JF
}

// Grid gradient of one (sample, plane) entry from its gradient row g (stage row l of G) and the
// tile texels: grid_sampler_2d_backward (generator.py:312-326 through ATen, border padding,
// align_corners) in the normalized cell,
//   gx = gxm sum_c g_c (s (T01 - T00) + n (T11 - T10)),  gy = gym sum_c g_c (e (T10 - T00) + w (T11 - T01))
// with T_yx the cell's texels (row y0 + y, column x0 + x), e = 1 - w, s = 1 - n, and the
// multipliers gxm / gym = (R-1)/2 strictly inside, else 0 (record flags).  A border-clipped
// point (x0 = R-1, w = 0, gxm = 0) normalized to (R-2, w = 1) gives the same gy, and likewise in y.
//
// NFI_TILE_GG 1 (default): the same sums as three channel dot products of first differences,
//   SA = sum_c g_c (T01 - T00),  SB = sum_c g_c (T11 - T10),  SC = sum_c g_c (T10 - T00),
//   gx = gxm (SA + n (SB - SA)),  gy = gym (SC + w (SB - SA))
// (s (T01 - T00) + n (T11 - T10) = A + n (B - A) and e (T10 - T00) + w (T11 - T01) = C + w (B - A),
// as T11 - T01 - T10 + T00 = B - A): per channel 3 differences + 3 FMAs on aligned register pairs
// (packed fp32, the float4 quads straight from the b128 reads) instead of ATen's 10 operations
// per channel with the cell weights broadcast into pairs (~30 register moves per quad pair).
// The differences are taken before any product, as ATen does; four partial sums per dot product
// (channel c mod 4) replace ATen's sequential channel order.  NFI_TILE_GG 0: ATen's form.
#ifndef NFI_TILE_GG
#define NFI_TILE_GG 1
#endif
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f4v pk_sub(f4v a, f4v b, float m1) {
  f4v r;
  r.xy = __builtin_elementwise_fma((f2v){b.x, b.y}, (f2v){m1, m1}, (f2v){a.x, a.y});
  r.zw = __builtin_elementwise_fma((f2v){b.z, b.w}, (f2v){m1, m1}, (f2v){a.z, a.w});
  return r;
}
#ifndef NFI_TILE_GG_UNROLL
#define NFI_TILE_GG_UNROLL 2
#endif
// dpc layout: NFI_DPC_PLANAR 1 (default) [3 planes][nsamp][2] — a chunk's entries (one plane,
// runs of consecutive samples) write consecutive 8-B pairs; 0: [nsamp][3][2] (each entry's pair
// 24 B apart, three tile passes' partial writes per line)
#ifndef NFI_DPC_PLANAR
#define NFI_DPC_PLANAR 1
#endif
__device__ __forceinline__ long long dpc_at(long long s, int q, long long nsamp) {
  return NFI_DPC_PLANAR ? ((long long)q * nsamp + s) * 2 : (s * 3 + q) * 2;
}
__device__ __forceinline__ void entry_grid_grad(const float* __restrict__ G, const float* __restrict__ Tex,
                                                int l, int4 rec, int q, float half, float* __restrict__ dpc,
                                                long long nsamp) {
  const int slot = rec.y & 31;
  const float w = __int_as_float(rec.z), n = __int_as_float(rec.w);
  float gx = 0.f, gy = 0.f;
  const float* tb = Tex + tex_at(slot);
#if NFI_TILE_GG
  f4v SA = {0.f, 0.f, 0.f, 0.f}, SB = SA, SC = SA;
  // -1 from an SGPR the compiler cannot see through: a - b as fma(b, -1, a) (one rounding, the
  // same value) stays a packed v_pk_fma_f32; hipcc scalarises a packed fsub into four v_sub_f32
  float m1;
  asm("s_mov_b32 %0, -1.0" : "=s"(m1));
#pragma unroll NFI_TILE_GG_UNROLL
  for (int k = 0; k < NC / 4; ++k) {
    const f4v g4 = *reinterpret_cast<const f4v*>(G + stage_q(l, k));
    const float* t = tb + 4 * k;
    const f4v t00 = *reinterpret_cast<const f4v*>(t);
    const f4v t01 = *reinterpret_cast<const f4v*>(t + XS);
    const f4v t10 = *reinterpret_cast<const f4v*>(t + TEXR);
    const f4v t11 = *reinterpret_cast<const f4v*>(t + TEXR + XS);
    SA += g4 * pk_sub(t01, t00, m1);
    SB += g4 * pk_sub(t11, t10, m1);
    SC += g4 * pk_sub(t10, t00, m1);
  }
  const float sa = (SA.x + SA.y) + (SA.z + SA.w), sb = (SB.x + SB.y) + (SB.z + SB.w);
  const float sc = (SC.x + SC.y) + (SC.z + SC.w);
  gx = fmaf(n, sb - sa, sa);
  gy = fmaf(w, sb - sa, sc);
#else
  const float e = 1.f - w, s = 1.f - n;
#pragma unroll 2
  for (int k = 0; k < NC / 4; ++k) {
    const float4 g4 = *reinterpret_cast<const float4*>(G + stage_q(l, k));
    const float* t = tb + 4 * k;
    const float4 t00 = *reinterpret_cast<const float4*>(t);
    const float4 t01 = *reinterpret_cast<const float4*>(t + XS);
    const float4 t10 = *reinterpret_cast<const float4*>(t + TEXR);
    const float4 t11 = *reinterpret_cast<const float4*>(t + TEXR + XS);
#define NFI_GG(C)                                                     \
  gx = fmaf(g4.C, fmaf(s, t01.C - t00.C, n * (t11.C - t10.C)), gx);   \
  gy = fmaf(g4.C, fmaf(e, t10.C - t00.C, w * (t11.C - t01.C)), gy);
    NFI_GG(x) NFI_GG(y) NFI_GG(z) NFI_GG(w)
#undef NFI_GG
  }
#endif
  const float2 out = make_float2((rec.y & 0x100) ? gx * half : 0.f, (rec.y & 0x200) ? gy * half : 0.f);
#if NFI_TILE_CHECK
  if (rec.x < 0 || rec.x >= nsamp) return;   // (code 3 counts it; never store out of range)
#endif
  *reinterpret_cast<float2*>(dpc + dpc_at(rec.x, q, nsamp)) = out;
}

// One workgroup-chunk c (< meta[0]) of a tile's entries; lds: TILE_LDS floats.
__device__ __forceinline__ void tile_chunk(const TileArgs& A, float* __restrict__ lds, int c) {
  const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), l = lane_id();
  const int h = l >> 5, cl = l & 31;
  float* G = lds + wv * TROWS;
  float* Tex = lds + 4 * TROWS;
  // half 0 weights row ly by (1 - n), half 1 row ly + 1 by n
  const float wsgn = h ? 1.f : -1.f, woff = h ? 0.f : 1.f;
  NFI_STAMP_INIT
  {
    // (wave-uniform scalars: readfirstlane keeps the entry loop's control and the register-image
    // index in SGPRs)
    const int tile = __builtin_amdgcn_readfirstlane(A.chunk_tile[c]);
#if NFI_TILE_CHECK
    if (tid == 0) {
      NFI_TCHK(c >= 0 && c < A.meta[0] && tile >= 0 && tile < A.K, 1, c, tile, 0, c, A.meta[0]);
    }
    if (tile < 0 || tile >= A.K) return;
#endif
    const int first = __builtin_amdgcn_readfirstlane(A.offsets[tile] + (c - A.chunk_start[tile]) * CHUNK);
    const int last = __builtin_amdgcn_readfirstlane(min(A.offsets[tile] + A.counts[tile], first + CHUNK));
#if NFI_TILE_CHECK
    if (tid == 0) {
      NFI_TCHK(first >= A.offsets[tile] && first < last && A.offsets[tile] + A.counts[tile] <= A.offsets[A.K],
               1, c, tile, 0, first, last);
      NFI_TCHK(A.cursor[tile] == A.offsets[tile] + A.counts[tile], 2, c, tile, 0, A.cursor[tile],
               A.offsets[tile] + A.counts[tile]);
    }
#endif
    int b, q, tx, ty;
    tile_decode(tile, A.tg, b, q, tx, ty);
    const float* src = A.planes + (long long)b * A.sb + (long long)q * A.sq;
    if (A.dpc) {
      // the tile's texels of plane q (texels past the plane edge are never referenced: cells
      // are normalized to x0, y0 <= R-2)
      for (int k = tid; k < TTX * TTY * (NC / 4); k += 256) {
        const int texel = k / (NC / 4), c4 = k % (NC / 4);
        const int gy = ty * TSY + texel / TTX, gx = tx * TSX + texel % TTX;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gy < A.R && gx < A.R) v = *reinterpret_cast<const float4*>(src + (long long)(gy * A.R + gx) * A.st + 4 * c4);
        *reinterpret_cast<float4*>(Tex + tex_at(texel) + 4 * c4) = v;
      }
      __syncthreads();
    }
#if NFI_TILE_CHECK
    // code 8 / 11: the staged texels read back against the planes (k = 8: after staging, 11: at
    // the end of the chunk's entry loops)
#define NFI_TEX_VERIFY(CODE)                                                                          \
    if (A.dpc) {                                                                                      \
      for (int k = tid; k < TTX * TTY * (NC / 4); k += 256) {                                         \
        const int texel = k / (NC / 4), c4 = k % (NC / 4);                                            \
        const int gy = ty * TSY + texel / TTX, gx = tx * TSX + texel % TTX;                           \
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);                                                   \
        if (gy < A.R && gx < A.R) v = *reinterpret_cast<const float4*>(src + (long long)(gy * A.R + gx) * A.st + 4 * c4); \
        const float4 s = *reinterpret_cast<const float4*>(Tex + tex_at(texel) + 4 * c4);              \
        NFI_TCHK(s.x == v.x && s.y == v.y && s.z == v.z && s.w == v.w, CODE, c, tile, tid, texel, c4); \
      }                                                                                               \
    }
    NFI_TEX_VERIFY(8)
#endif
    const float half = (float)(A.R - 1) / 2.f;
    // each wave sums a contiguous quarter of the chunk (runs of one ray stay together)
    const int per = (((last - first) + 3) / 4 + 7) & ~7;
    const int b0 = first + wv * per, b1 = min(last, b0 + per);
    img32 img = 0.f;
    if (b0 < b1) {
      const cint4_p L = (cint4_p)A.list;
      // 8 entries per step.  Scalar (record) and LDS (row) loads share lgkmcnt and scalar loads
      // return out of order, so a step that waits for its LDS rows also waits for every scalar load
      // in flight: the next step's records are issued only after this step's rows have been
      // waited for (a consume + compiler barrier), into the other half of a ping-pong pair — the
      // one wait per step then covers a scalar load that had a whole step to arrive.  The surplus
      // entries of the last step read the next tile's records or the zeroed list padding
      // (chunk_map_kernel): valid cells, and their zeroed rows add 0.
#define NFI_ENTRY(R, K)                                                                              \
  tile_entry(img, __builtin_amdgcn_readfirstlane(R[K].y) & 31, __int_as_float(R[K].z), __int_as_float(R[K].w), \
             gv[K], wsgn, woff)
#if NFI_TILE_CHECK
      // code 6: each scalar record of the entry loop against the batch's vector record (lane U + k)
#define NFI_STEP_CHECK(U, RUSE)                                                                      \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) if ((U) + k < n) {                                 \
      const int vx = __shfl(crec.x, (U) + k), vy = __shfl(crec.y, (U) + k);                          \
      const int vz = __shfl(crec.z, (U) + k), vw = __shfl(crec.w, (U) + k);                          \
      NFI_TCHK(RUSE[k].x == vx && RUSE[k].y == vy && RUSE[k].z == vz && RUSE[k].w == vw, 6, c, tile, \
               (U) + k, RUSE[k].x, vx);                                                              \
    }
#else
#define NFI_STEP_CHECK(U, RUSE)
#endif
#define NFI_STEP(U, RUSE, RNEXT)                                                                     \
  {                                                                                                  \
    float gv[8];                                                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) gv[k] = G[stage_at((U) + k, cl)];                 \
    asm volatile("" ::"v"(gv[0]), "v"(gv[1]), "v"(gv[2]), "v"(gv[3]), "v"(gv[4]), "v"(gv[5]),       \
                 "v"(gv[6]), "v"(gv[7]) : "memory");                                                 \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) RNEXT[k] = L[base_ + (U) + 8 + k];                 \
    NFI_STEP_CHECK(U, RUSE)                                                                          \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) NFI_ENTRY(RUSE, k);                               \
  }
      // Rows loaded coalesced: lane l holds float4 (l & 7) of entry 8j + (l >> 3), j = 0..6 (the
      // entry's row index comes from its lane's record by ds_bpermute): each b128 load reads 8
      // whole 128-B rows instead of one 16-B piece of 56 different rows.
#if NFI_TILE_CHECK
      // codes 3 / 5: the shuffled row index against the record loaded directly; clamped into range
#define NFI_ROW_CHECK(J, RB)                                                                         \
    {                                                                                                \
      const int want_ = A.list[min((RB) + 8 * (J) + (l >> 3), b1 - 1)].x;                            \
      NFI_TCHK(row_ == want_, 5, c, tile, l, row_, want_);                                           \
      NFI_TCHK(row_ >= 0 && row_ < A.nsamp, 3, c, tile, l, row_, A.nsamp);                          \
      row_ = (row_ >= 0 && row_ < A.nsamp) ? row_ : 0;                                               \
    }
#else
#define NFI_ROW_CHECK(J, RB)
#endif
#define NFI_LD1(J, V, SX, RB)                                                                        \
  {                                                                                                  \
    int row_ = __shfl((SX), 8 * (J) + (l >> 3));                                                    \
    NFI_ROW_CHECK(J, RB)                                                                             \
    V = *reinterpret_cast<const float4*>(A.gfeat + (long long)row_ * NC + 4 * (l & 7));              \
  }
#define NFI_LOAD_ROWC(REC, RB)                                                                       \
  {                                                                                                  \
    const int sx_ = (REC).x;                                                                         \
    _Pragma("unroll") for (int j = 0; j < BATCH / 8; ++j) NFI_LD1(j, rc[j], sx_, RB)                 \
  }
#define NFI_ST1(J, V)                                                                                \
  {                                                                                                  \
    const int e_ = 8 * (J) + (l >> 3);                                                               \
    lds_st(reinterpret_cast<float4*>(G + e_ * XS + 4 * (l & 7)), e_ < n ? V : make_float4(0.f, 0.f, 0.f, 0.f)); \
  }
#if NFI_TILE_CHECK
      // code 7: the stored gradient rows read back; code 12 (after the entry loop): the rows
      // against gfeat itself; codes 3 / 4 / 10: the batch's records
#define NFI_G_VERIFY(CODE)                                                                           \
    _Pragma("unroll") for (int j = 0; j < BATCH / 8; ++j) {                                          \
      const int e_ = 8 * j + (l >> 3);                                                               \
      const float4 s_ = *reinterpret_cast<const float4*>(G + e_ * XS + 4 * (l & 7));                 \
      float4 w_ = make_float4(0.f, 0.f, 0.f, 0.f);                                                   \
      if (e_ < n) {                                                                                  \
        const int rx_ = A.list[base_ + e_].x;                                                        \
        if (rx_ >= 0 && rx_ < A.nsamp) w_ = *reinterpret_cast<const float4*>(A.gfeat + (long long)rx_ * NC + 4 * (l & 7)); \
      }                                                                                              \
      NFI_TCHK(s_.x == w_.x && s_.y == w_.y && s_.z == w_.z && s_.w == w_.w, CODE, c, tile, l, base_ + e_, j); \
    }
#define NFI_BATCH_CHECK()                                                                            \
    NFI_G_VERIFY(7)                                                                                  \
    if (l < n) {                                                                                     \
      const int4 d_ = A.list[base_ + l];                                                             \
      NFI_TCHK(d_.x == crec.x && d_.y == crec.y && d_.z == crec.z && d_.w == crec.w, 6, c, tile, l, crec.x, d_.x); \
      NFI_TCHK(crec.x >= 0 && crec.x < A.nsamp, 3, c, tile, l, crec.x, A.nsamp);                    \
      NFI_TCHK((crec.y & 31) <= 30 && (crec.y & ~0x31f) == 0, 4, c, tile, l, crec.y, 30);           \
      const float w_ = __int_as_float(crec.z), n_ = __int_as_float(crec.w);                          \
      NFI_TCHK(w_ >= 0.f && w_ <= 1.f && n_ >= 0.f && n_ <= 1.f, 10, c, tile, l, crec.z, crec.w);  \
    }
#define NFI_CREC(VREC) const int4 crec = VREC;
#else
#define NFI_BATCH_CHECK()
#define NFI_G_VERIFY(CODE)
#define NFI_CREC(VREC)
#endif
#define NFI_REC_FIRST()                                                                              \
    iv4 ra[8], rb[8];                                                                                \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) ra[k] = L[base_ + k];
#define NFI_NEXT_REC(VREC, AHEAD)                                                                    \
    VREC = vnext;                                                                                    \
    vnext = A.list[min(base_ + 2 * (AHEAD) + l, b1 - 1)];
#define NFI_BATCHC(BASE, VREC, AHEAD)                                                                \
  {                                                                                                  \
    const int base_ = (BASE);                                                                        \
    const int n = min(BATCH, b1 - base_);                                                            \
    _Pragma("unroll") for (int j = 0; j < BATCH / 8; ++j) NFI_ST1(j, rc[j])                         \
    wave_lds_sync();                                                                                 \
    NFI_CREC(VREC)                                                                                   \
    NFI_BATCH_CHECK()                                                                                \
    if (A.dpc && l < n) entry_grid_grad(G, Tex, l, VREC, q, half, A.dpc, A.nsamp);                   \
    NFI_NEXT_REC(VREC, AHEAD)                                                                        \
    NFI_LOAD_ROWC(VREC, base_ + (AHEAD))                                                             \
    NFI_STAMP(24)                                                                                    \
    NFI_REC_FIRST()                                                                                  \
    for (int u = 0; u < n; u += 16) {                                                                \
      NFI_STEP(u, ra, rb)                                                                            \
      if (u + 8 >= n) break;                                                                         \
      NFI_STEP(u + 8, rb, ra)                                                                        \
    }                                                                                                \
    NFI_G_VERIFY(12)                                                                                 \
    wave_lds_sync();                                                                                 \
    NFI_STAMP(25)                                                                                    \
  }
      static_assert(BATCH % 8 == 0, "coalesced row loads of 8 entries each");
      float4 rc[BATCH / 8];
      int4 vrec = A.list[min(b0 + l, b1 - 1)];
      // the next batch's records are already in registers when its rows are issued (the row
      // loads do not wait a record round trip)
      int4 vnext = A.list[min(b0 + BATCH + l, b1 - 1)];
      NFI_LOAD_ROWC(vrec, b0)
      for (int bb = b0; bb < b1; bb += BATCH) NFI_BATCHC(bb, vrec, BATCH)
#undef NFI_BATCHC
#undef NFI_NEXT_REC
#undef NFI_REC_FIRST
#undef NFI_ST1
#undef NFI_LOAD_ROWC
#undef NFI_LD1
#undef NFI_STEP
#undef NFI_ENTRY
#undef NFI_STEP_CHECK
#undef NFI_ROW_CHECK
#undef NFI_BATCH_CHECK
#undef NFI_G_VERIFY
#undef NFI_CREC
    }
    NFI_STAMP(26)
#if NFI_TILE_CHECK
    NFI_TEX_VERIFY(11)
#undef NFI_TEX_VERIFY
#endif
    __syncthreads();   // every wave is done with its row stage
    // wave images -> LDS [wave][half][slot][channel]
#pragma unroll
    for (int r = 0; r < 32; ++r) lds[wv * 2048 + (h * 32 + r) * NC + cl] = img[r];
    __syncthreads();
#if NFI_TILE_CHECK
    // code 9: the dumped wave images read back
#pragma unroll
    for (int r = 0; r < 32; ++r) NFI_TCHK(lds[wv * 2048 + (h * 32 + r) * NC + cl] == img[r], 9, c, tile, l, r, wv);
#endif
    float* dq = A.dplanes + (long long)b * A.sb + (long long)q * A.sq;
    for (int k = tid; k < TTX * TTY * NC; k += 256) {
      const int texel = k / NC, ch = k % NC;
      const int yl = texel / TTX, xl = texel % TTX;
      float v = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const float* im = lds + w4 * 2048;
        if (yl < TSY) v += im[(yl * TTX + xl) * NC + ch];
        if (yl >= 1) v += im[(32 + (yl - 1) * TTX + xl) * NC + ch];
      }
      const int gy = ty * TSY + yl, gx = tx * TSX + xl;
      if (A.part) A.part[(long long)c * (TTX * TTY * NC) + k] = v;
      else if (v != 0.f && gy < A.R && gx < A.R) unsafeAtomicAdd(dq + (gy * A.R + gx) * A.st + ch, v);
    }
#if NFI_TILE_CHECK
    // the second sum of d planes (compared with the first by tile_shadow_compare_kernel): every
    // entry of this wave's range again, straight from the list and gfeat in global memory, one
    // float atomic per (entry, texel, channel) — no LDS stage, scalar records, register image or dump
    if (A.shadow) {
      float* sq_ = A.shadow + (long long)b * A.sb + (long long)q * A.sq;
      for (int e = b0; e < b1; ++e) {
        const int4 r_ = A.list[e];
        if (r_.x < 0 || r_.x >= A.nsamp) continue;
        const int slot = r_.y & 31, ly = slot / TTX, lx = slot % TTX;
        const float w = __int_as_float(r_.z), nn = __int_as_float(r_.w);
        const float g = A.gfeat[(long long)r_.x * NC + cl] * (h ? nn : 1.f - nn);
        const int gy = ty * TSY + ly + h, gx = tx * TSX + lx;
        if (gy < A.R && gx + 1 < A.R) {
          unsafeAtomicAdd(sq_ + (gy * A.R + gx) * A.st + cl, g * (1.f - w));
          unsafeAtomicAdd(sq_ + (gy * A.R + gx + 1) * A.st + cl, g * w);
        }
      }
    }
#endif
    __syncthreads();
    NFI_STAMP(27)
  }
}

// ---------------------------------------------------------------------------------------
// Eval outputs of render() (run.py:227-257, 293-335), one wave per ray from the forward's saved
// state: compositing weights w_i in merged order (the forward's arithmetic), then
//   semantics  sum_i w_i softmax(logits_i)                    (generator.py:672-674)
//   coords     sum_i w_i (ro + rd t_i)                        (generator.py:643-644)
//   normals    sum_i w_i normalize(d sdf_i / d p_i) (+ 1-mask on white) (generator.py:599-622,
//              nerf_utils.py:146-161): d sdf / d features by the MFMA decoder backward with
//              dY = e_0, then the tap derivative by a re-gather with a per-point reduction.
// Forward-only (the reference's callers of these outputs render without gradients).
// ---------------------------------------------------------------------------------------
template <int NPL, int NOUT>
__global__ void __launch_bounds__(256) extras_kernel(nfi_render_args a) {
  __shared__ __attribute__((aligned(16))) float lds[4 * (XTILE + 256)];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= nrays) return;
  float* X = lds + wv * (XTILE + 256);
  float* ND = X + XTILE;   // [64][4] per-point d sdf / d p
  const int N = a.fine ? 2 * a.S : a.S;
  const float sr = a.field.scene_range;
  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};
  float t[NPL], w[NPL];
  float sm = 0.f;
  {
    float al[NPL], aa[NPL], T[NPL];
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      const int i = e * 64 + l;
      const bool v = i < N;
      t[e] = v ? a.t_saved[r * N + i] : 0.f;
      const float sg = v ? a.sigma_saved[r * N + i] : 0.f;
      const float dist = (i < N - 1) ? fmul(fsub(a.t_saved[r * N + i + 1], t[e]), R.rdn) : 0.f;
      float ex;
      alpha_of(sg, dist, al[e], aa[e], ex);
      if (!v) {
        al[e] = 0.f;
        aa[e] = 1.f;
      }
    }
    excl_prod<NPL>(aa, T);
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      w[e] = (e * 64 + l < N) ? fmul(al[e], T[e]) : 0.f;
      sm += w[e];
    }
  }
  const float mask = wave_sum(sm);
  if (a.extras & 4) {
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      if (e * 64 + l < N) {
        c0 = fmaf(w[e], fadd(R.o[0], fmul(R.d[0], t[e])), c0);
        c1 = fmaf(w[e], fadd(R.o[1], fmul(R.d[1], t[e])), c1);
        c2 = fmaf(w[e], fadd(R.o[2], fmul(R.d[2], t[e])), c2);
      }
    }
    c0 = wave_sum(c0);
    c1 = wave_sum(c1);
    c2 = wave_sum(c2);
    if (l == 0) {
      a.semantic_map[r * 3 + 0] = c0;
      a.semantic_map[r * 3 + 1] = c1;
      a.semantic_map[r * 3 + 2] = c2;
    }
  } else if (a.extras & 2) {
    float acc[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] = 0.f;
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      const int i = e * 64 + l;
      if (i < N) {
        const int ei = a.perm[r * N + i];
        float y[NA];
        if constexpr (NOUT == NOV) {
          // logits of the view-direction mapper closure (generator.py:661-663, 672-674)
          float yv[NOV], y11[NO];
#pragma unroll
          for (int k = 0; k < NOV; ++k) yv[k] = a.y_saved[r * NOV * N + k * N + ei];
          viewdir_head_in(yv, a.field.xray + r * NVF, a.field.vhead, a.field.vhead_out, y11);
#pragma unroll
          for (int k = 0; k < NA; ++k) y[k] = y11[1 + k];
        } else {
#pragma unroll
          for (int k = 0; k < NA; ++k) y[k] = a.y_saved[r * NO * N + (1 + k) * N + ei];
        }
        // softmax as head_forward forms it
        float m = y[0];
#pragma unroll
        for (int k = 1; k < NA; ++k) m = fmaxf(m, y[k]);
        float p[NA], sum = 0.f;
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          p[k] = __expf(y[k] - m);
          sum += p[k];
        }
        const float rs = 1.f / sum;
#pragma unroll
        for (int k = 0; k < NA; ++k) acc[k] = fmaf(w[e], p[k] * rs, acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const float v = wave_sum(acc[k]);
      if (l == 0) a.semantic_map[r * NA + k] = v;
    }
  }
  if (a.extras & 1) {
    float n0 = 0.f, n1 = 0.f, n2 = 0.f;
    const int j16 = l & 15, q = l >> 4;
    const int sub = l >> 4, dx = (l >> 3) & 1, q4 = l & 7;
#pragma unroll 1
    for (int e = 0; e < NPL; ++e) {
      if (e * 64 >= N) break;
      const int npts = min(64, N - e * 64);
      // d sdf / d x for the chunk's points: decoder backward with dY = e_0 on the matrix cores
      f4v xa[4], xb[4];
#pragma unroll
      for (int sb = 0; sb < 4; ++sb) {
        const int ip = e * 64 + 16 * sb + j16;
        xa[sb] = f4v{0.f, 0.f, 0.f, 0.f};
        xb[sb] = xa[sb];
        if (ip < N) {
          const float* xr = a.x_saved + (r * N + (int)a.perm[r * N + ip]) * NC + 8 * q;
          xa[sb] = ld4(xr);
          xb[sb] = ld4(xr + 4);
        }
      }
      // dY rows: the unit vector of the distance output
      wave_lds_sync();
      {
        float dyr[DYC<NOUT>];
#pragma unroll
        for (int o = 0; o < DYC<NOUT>; ++o) dyr[o] = (o == 0) ? 1.f : 0.f;
        lds_store_keep(X + l * XS, dyr);
      }
      wave_lds_sync();
      f4v gxo[2][4];
      mlp_backward<NOUT>(a.field.dec, xa, xb, X, 1.f / 3.f, [&](int cb, int sb, f4v gv) { gxo[cb][sb] = gv; });
      wave_lds_sync();
#pragma unroll
      for (int sb = 0; sb < 4; ++sb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          lds_st(reinterpret_cast<f4v*>(X + (16 * sb + j16) * XS + 16 * cb + 4 * q), gxo[cb][sb]);
      wave_lds_sync();
      // tap derivative per point (quad layout), reduced over the point's 16 lanes
      PointP P;
      point_params(R.o, R.d, (e * 64 + l < N) ? t[e] : R.near_, sr, pv.R, P);
      const int ngrp = (npts + 3) >> 2;
#pragma unroll 1
      for (int gi = 0; gi < ngrp; ++gi) {
        const int j = 4 * gi + sub;
        const float4 gv = *reinterpret_cast<const float4*>(X + j * XS + 4 * q4);
        float GX[3], GY[3];
#pragma unroll
        for (int pq = 0; pq < 3; ++pq) {
          const int pk = __shfl(P.pl[pq].tex, j);
          const float e_ = __shfl(P.pl[pq].e, j), ww = __shfl(P.pl[pq].w, j);
          const float s = __shfl(P.pl[pq].s, j), n = __shfl(P.pl[pq].n, j);
          const float gxm = __shfl(P.pl[pq].gxm, j), gym = __shfl(P.pl[pq].gym, j);
          const int t0 = (pk & 0xFFFFF) + (dx ? ((pk >> 20) & 1) : 0);
          const int t1 = t0 + (((pk >> 21) & 1) ? pv.R : 0);
          const float* b = pv.base + pq * pv.sq + 4 * q4;
          const float4 v0 = *reinterpret_cast<const float4*>(b + t0 * pv.st);
          const float4 v1 = *reinterpret_cast<const float4*>(b + t1 * pv.st);
          const float wx = dx ? ww : e_;
          const float ax = (s * v0.x + n * v1.x) * gv.x + (s * v0.y + n * v1.y) * gv.y +
                           (s * v0.z + n * v1.z) * gv.z + (s * v0.w + n * v1.w) * gv.w;
          const float ay = (v1.x - v0.x) * gv.x + (v1.y - v0.y) * gv.y + (v1.z - v0.z) * gv.z +
                           (v1.w - v0.w) * gv.w;
          GX[pq] = (dx ? ax : -ax) * gxm;
          GY[pq] = wx * ay * gym;
        }
        float d0 = GX[0] + GX[1], d1 = GY[0] + GX[2], d2 = GY[1] + GY[2];
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          d0 += __shfl_xor(d0, m);
          d1 += __shfl_xor(d1, m);
          d2 += __shfl_xor(d2, m);
        }
        if ((l & 15) == 0) {
          ND[j * 4 + 0] = d0;
          ND[j * 4 + 1] = d1;
          ND[j * 4 + 2] = d2;
        }
      }
      wave_lds_sync();
      if (e * 64 + l < N) {
        // x = p / scene_range: d sdf / d p = (d sdf / d x) / scene_range; F.normalize (eps 1e-12)
        const float g0 = ND[l * 4 + 0] / sr, g1 = ND[l * 4 + 1] / sr, g2 = ND[l * 4 + 2] / sr;
        const float nr = fmaxf(tnorm3(g0, g1, g2), 1e-12f);
        n0 = fmaf(w[e], g0 / nr, n0);
        n1 = fmaf(w[e], g1 / nr, n1);
        n2 = fmaf(w[e], g2 / nr, n2);
      }
      wave_lds_sync();
    }
    n0 = wave_sum(n0);
    n1 = wave_sum(n1);
    n2 = wave_sum(n2);
    if (l == 0) {
      const float bg = a.white_bg ? fsub(1.f, mask) : 0.f;
      a.normal_map[r * 3 + 0] = n0 + bg;
      a.normal_map[r * 3 + 1] = n1 + bg;
      a.normal_map[r * 3 + 2] = n2 + bg;
    }
  }
}

// d planes and the per-(sample, plane) grid gradients of the pose path: a grid of at most
// TILE_WGS workgroups takes the chunks IN KEY ORDER from a queue (one atomic per chunk on
// meta[1], zeroed before the launch), so the chunks in flight at any time are those of one or
// two beams (tile_grid) whatever the hardware's dispatch order, and a chunk-count bound of
// 10^5..10^6 mostly empty tiles costs no empty workgroups.  Every workgroup leaves when the
// queue passes meta[0].  (Replaces an XCD-grouped static chunk order, measured no faster.)
#ifndef NFI_TILE_OCC
#define NFI_TILE_OCC 4
#endif
constexpr int TILE_WGS = 2048;   // >= 256 CUs x NFI_TILE_OCC workgroups resident
#ifndef NFI_TILE_REV
#define NFI_TILE_REV 0   // 1: last key first (the beams the field backward wrote last)
#endif
#if NFI_TILE_CHECK
// sum over d planes of (d planes - snapshot - shadow)^2 and shadow^2 (the tile pass's added d planes
// against the per-entry atomics of the same entries), into two doubles
__global__ void __launch_bounds__(256) tile_shadow_compare_kernel(const float* __restrict__ dp, const float* __restrict__ snap,
                                                                  const float* __restrict__ sh, long long n, double* out) {
  double d2 = 0.0, s2 = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double d = (double)dp[i] - (double)snap[i] - (double)sh[i];
    d2 += d * d;
    s2 += (double)sh[i] * (double)sh[i];
  }
  for (int m = 32; m >= 1; m >>= 1) {
    d2 += __shfl_xor(d2, m);
    s2 += __shfl_xor(s2, m);
  }
  if (lane_id() == 0) {
    atomicAdd(out, d2);
    atomicAdd(out + 1, s2);
  }
}
#endif

__global__ void __launch_bounds__(256, NFI_TILE_OCC) tile_kernel(TileArgs A) {
  __shared__ __attribute__((aligned(16))) float lds[TILE_LDS];
  __shared__ int next;
  const int M = A.meta[0];
  for (;;) {
    if (threadIdx.x == 0) next = atomicAdd(A.meta + 1, 1);
    __syncthreads();
    const int k = next;
    __syncthreads();   // (every lane has read it before lane 0 takes the next one)
    if (k >= M) return;
    tile_chunk(A, lds, NFI_TILE_REV ? M - 1 - k : k);
  }
}

// Ray-coordinate gradients from the tile pass's grid gradients, one wave per 64 merged samples:
// dL/dp_j = (gx_xy + gx_xz, gy_xy + gx_yz, gy_xz + gy_yz)_j / scene_range (planes xy, xz, yz take
// coordinates (x, y), (x, z), (y, z); generator.py:312-326, 604), dL/d ro = sum_j dL/dp_j and
// dL/d rd = sum_j t_j dL/dp_j (p = ro + rd t, run.py:283-288).  Samples outside the box have no
// entries (their sigma and weight are 0, so their feature gradient is exactly zero).
// One wave per ray over its NPL chunks of 64 (no atomics: composite_bwd_kernel wrote g_ro / g_rd
// earlier on the stream, this wave owns the ray's six sums and adds them in place).
template <int NPL>
__global__ void __launch_bounds__(256) dcoord_reduce_kernel(nfi_render_args a, BwdArgs g, const float* __restrict__ dpc) {
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = ray_of_block(blockIdx.x, 4, a) + wv;
  if (r >= nrays) return;
  const int N = a.fine ? 2 * a.S : a.S;
  const float sr = a.field.scene_range;
  RayCtx R;
  load_ray(a, r, R);
  // every load at a clamped index, issued together (the grid-gradient row of a dead sample is
  // never written: whatever it holds is dropped by the select)
  float ts[NPL];
  float2 xy[NPL], xz[NPL], yz[NPL];
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const int ic = min(e * 64 + l, N - 1);
    ts[e] = a.t_saved[r * N + ic];
    const long long si = r * N + ic, ns = nrays * N;
    xy[e] = *reinterpret_cast<const float2*>(dpc + dpc_at(si, 0, ns));
    xz[e] = *reinterpret_cast<const float2*>(dpc + dpc_at(si, 1, ns));
    yz[e] = *reinterpret_cast<const float2*>(dpc + dpc_at(si, 2, ns));
  }
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll
  for (int e = 0; e < NPL; ++e) {
    const bool v = e * 64 + l < N;
    const float te = v ? ts[e] : R.near_;
    // the in-box test of point_params (the tile entries were made with the same arithmetic)
    float cx[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) cx[k] = fdiv(fadd(R.o[k], fmul(R.d[k], te)), sr);
    const bool live = v && !(fabsf(cx[0]) > 1.f || fabsf(cx[1]) > 1.f || fabsf(cx[2]) > 1.f);
    const float d0 = live ? xy[e].x + xz[e].x : 0.f;
    const float d1 = live ? xy[e].y + yz[e].x : 0.f;
    const float d2 = live ? xz[e].y + yz[e].y : 0.f;
    s0 += d0;
    s1 += d1;
    s2 += d2;
    u0 = fmaf(d0, te, u0);
    u1 = fmaf(d1, te, u1);
    u2 = fmaf(d2, te, u2);
  }
  const float gro0 = wave_sum(s0) / sr, gro1 = wave_sum(s1) / sr, gro2 = wave_sum(s2) / sr;
  const float grd0 = wave_sum(u0) / sr, grd1 = wave_sum(u1) / sr, grd2 = wave_sum(u2) / sr;
  if (l < 3) {
    const float ro = l == 0 ? gro0 : (l == 1 ? gro1 : gro2);
    const float rd = l == 0 ? grd0 : (l == 1 ? grd1 : grd2);
    g.g_ro[r * 3 + l] += ro;
    g.g_rd[r * 3 + l] += rd;
  }
}

// =======================================================================================
// Per-stage seams: the nerf_utils functions and the sampler closure as launches
// of their own, for callers that use one of them without the fused render.  They reuse the
// fused kernels' device functions (tap gather, decoder on the matrix cores, heads, fp64 wave
// scans, the compositing suffix scan) and the same rounding order.
// =======================================================================================

// ---- sample_pdf (nerf_utils.py:185-224): bins [n][NB], weights [n][NB-1] -> [n][S] ----------
// One wave per ray: CDF in the wave's LDS slice (fp64 scan), one binary search per sample.
constexpr int PDF_NBMAX = 1024;
__global__ void __launch_bounds__(256) sample_pdf_kernel(const float* __restrict__ bins,
                                                         const float* __restrict__ weights, long long n, int NB,
                                                         int S, int deterministic, const float* __restrict__ u,
                                                         unsigned long long seed, unsigned long long offset,
                                                         float* __restrict__ out) {
  __shared__ float lds[4 * 2 * PDF_NBMAX];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  float* cdf = lds + wv * 2 * PDF_NBMAX;
  float* bn = cdf + PDF_NBMAX;
  const int NW = NB - 1;
  const float* w = weights + r * NW;
  // weights + 1e-5, normalised by their sum (float, ATen's order), cumsum (accumulated in fp64 as
  // ATen's CPU cumsum does); the padded weights are staged in the bins' half of the slice
  for (int i = l; i < NW; i += 64) bn[i] = fadd(w[i], 1e-5f);
  wave_lds_sync();
  const float totf = aten_sum_f32(bn, NW);
  double carry = 0.0;
  for (int c = 0; c < NW; c += 64) {
    const int i = c + l;
    const float pdf = (i < NW) ? fdiv(bn[min(i, NW - 1)], totf) : 0.f;
    const double inc = wave_incl_sum_d((double)pdf) + carry;
    if (i < NW) cdf[i + 1] = (float)inc;
    carry = readlane(inc, 63);
  }
  wave_lds_sync();
  for (int i = l; i < NB; i += 64) bn[i] = bins[r * NB + i];
  if (l == 0) cdf[0] = 0.f;
  wave_lds_sync();
  for (int c = 0; c < S; c += 64) {
    const int i = c + l;
    if (i >= S) break;
    const float uu = deterministic ? tlinspace01(i, S) : (u ? u[r * S + i] : rng_uniform(seed, offset, r, i, 1));
    int lo = 0, hi = NB;          // searchsorted(cdf, u, right=True): entries <= u
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (cdf[m] <= uu) lo = m + 1;
      else hi = m;
    }
    const int below = max(0, lo - 1), above = min(NB - 1, lo);
    const float c0 = cdf[below], c1 = cdf[above];
    const float b0 = bn[below], b1 = bn[above];
    float denom = fsub(c1, c0);
    denom = (denom < 1e-5f) ? 1.f : denom;
    const float tt = fdiv(fsub(uu, c0), denom);
    out[r * S + i] = fadd(b0, fmul(tt, fsub(b1, b0)));
  }
}

// ---- render_volume_density (nerf_utils.py:125-163) on caller samples ------------------------
// sigma [n][N], rgb [n][N][3], rd [n][3] (its norm scales the distances), t [n][N] ->
// rgb_map [n][3] (+ 1 - mask with a white background), depth [n], mask [n], weights [n][N]
// (optional).  One wave per ray; chunks of 64 samples with the fp64 transmittance carried.
constexpr int COMP_NMAX = 1024;
__global__ void __launch_bounds__(256) composite_fwd_kernel(const float* __restrict__ sigma,
                                                            const float* __restrict__ rgb,
                                                            const float* __restrict__ rd,
                                                            const float* __restrict__ tv, long long n, int N,
                                                            int white, float* __restrict__ rgb_map,
                                                            float* __restrict__ depth, float* __restrict__ mask,
                                                            float* __restrict__ wts) {
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  const float rdn = tnorm3(rd[r * 3 + 0], rd[r * 3 + 1], rd[r * 3 + 2]);
  const float* t = tv + r * N;
  double carry = 1.0;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, sm = 0.f, sd = 0.f;
  for (int c = 0; c < N; c += 64) {
    const int i = c + l;
    const int ic = min(i, N - 1);
    const float ti = t[ic], tn = t[min(i + 1, N - 1)], sg = sigma[r * N + ic];
    // (rgb NULL: the weights only, render_volume_density_weights_only)
    const float c0 = rgb ? rgb[(r * N + ic) * 3 + 0] : 0.f, c1 = rgb ? rgb[(r * N + ic) * 3 + 1] : 0.f;
    const float c2 = rgb ? rgb[(r * N + ic) * 3 + 2] : 0.f;
    const float dist = (i < N - 1) ? fmul(fsub(tn, ti), rdn) : 0.f;
    float al, aa, ex;
    alpha_of(i < N ? sg : 0.f, dist, al, aa, ex);
    al = i < N ? al : 0.f;
    aa = i < N ? aa : 1.f;
    const double inc = wave_incl_prod_d((double)aa);
    const double exc = dpp_fill<0x138>(inc, 1.0);
    const float T = (float)(carry * exc);
    carry = carry * readlane(inc, 63);
    const float w = fmul(al, T);
    if (i < N) {
      s0 = fmaf(w, c0, s0);
      s1 = fmaf(w, c1, s1);
      s2 = fmaf(w, c2, s2);
      sm += w;
      sd = fmaf(w, ti, sd);
      if (wts) wts[r * N + i] = w;
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  sm = wave_sum(sm);
  sd = wave_sum(sd);
  if (l == 0 && rgb_map) {
    const float bg = white ? fsub(1.f, sm) : 0.f;
    rgb_map[r * 3 + 0] = s0 + bg;
    rgb_map[r * 3 + 1] = s1 + bg;
    rgb_map[r * 3 + 2] = s2 + bg;
    mask[r] = sm;
    depth[r] = sd;
  }
}

// Backward: dL/d rgb_map [n][3], dL/d mask [n] and optionally dL/d weights [n][N] (maps the
// caller built on the weights output) -> d sigma [n][N], d rgb [n][N][3], and optionally
// d rd [n][3] (through ||rd||) and d t [n][N] (through the distances; the reference's depth values
// carry no gradient inside render(), but a caller's may).  The reverse affine scan of
// composite_bwd_kernel (suffix_affine), the transmittance of the forward recomputed into LDS.
__global__ void __launch_bounds__(256) composite_bwd_seam_kernel(
    const float* __restrict__ sigma, const float* __restrict__ rgb, const float* __restrict__ rd,
    const float* __restrict__ tv, long long n, int N, int white, const float* __restrict__ g_rgb,
    const float* __restrict__ g_mask, const float* __restrict__ g_w, float* __restrict__ d_sigma,
    float* __restrict__ d_rgb, float* __restrict__ d_rd, float* __restrict__ d_t) {
  __shared__ float lds[4 * 2 * COMP_NMAX];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  float* LT = lds + wv * 2 * COMP_NMAX;   // transmittance T_i
  float* LG = LT + COMP_NMAX;             // dL/d dist_i (for d t)
  const float d0 = rd[r * 3 + 0], d1 = rd[r * 3 + 1], d2 = rd[r * 3 + 2];
  const float rdn = tnorm3(d0, d1, d2);
  const float* t = tv + r * N;
  double carry = 1.0;
  for (int c = 0; c < N; c += 64) {
    const int i = c + l;
    const int ic = min(i, N - 1);
    const float dist = (i < N - 1) ? fmul(fsub(t[min(i + 1, N - 1)], t[ic]), rdn) : 0.f;
    float al, aa, ex;
    alpha_of(i < N ? sigma[r * N + ic] : 0.f, dist, al, aa, ex);
    aa = i < N ? aa : 1.f;
    const double inc = wave_incl_prod_d((double)aa);
    const double exc = dpp_fill<0x138>(inc, 1.0);
    if (i < N) LT[i] = (float)(carry * exc);
    carry = carry * readlane(inc, 63);
  }
  wave_lds_sync();
  // (g_rgb / g_mask NULL: zero — the weights-only seam)
  const float gr0 = g_rgb ? g_rgb[r * 3 + 0] : 0.f, gr1 = g_rgb ? g_rgb[r * 3 + 1] : 0.f;
  const float gr2 = g_rgb ? g_rgb[r * 3 + 2] : 0.f;
  const float gm = (g_mask ? g_mask[r] : 0.f) - (white ? (gr0 + gr1 + gr2) : 0.f);
  float grdn = 0.f, cB = 0.f;
  const int nch = (N + 63) / 64;
  for (int ch = nch - 1; ch >= 0; --ch) {
    const int i = ch * 64 + l;
    const bool v = i < N;
    const int ic = min(i, N - 1);
    const float raw = (i < N - 1) ? fsub(t[min(i + 1, N - 1)], t[ic]) : 0.f;
    const float dist = fmul(raw, rdn);
    const float sg = v ? sigma[r * N + ic] : 0.f;
    float al, aa, ex;
    alpha_of(sg, dist, al, aa, ex);
    al = v ? al : 0.f;
    aa = v ? aa : 1.f;
    const float c0 = rgb ? rgb[(r * N + ic) * 3 + 0] : 0.f, c1 = rgb ? rgb[(r * N + ic) * 3 + 1] : 0.f;
    const float c2 = rgb ? rgb[(r * N + ic) * 3 + 2] : 0.f;
    const float gwx = (g_w && v) ? g_w[r * N + ic] : 0.f;
    const float ee = v ? (gr0 * c0 + gr1 * c1 + gr2 * c2) + gm + gwx : 0.f;
    const float T = v ? LT[ic] : 0.f;
    const float Sk = suffix_affine(aa, ee * al, cB);
    const float dal = T * (ee - Sk);              // dL/d alpha_i
    const float gdist = dal * sg * ex;            // dL/d dist_i (d alpha / d dist = sigma exp(-sigma dist))
    grdn += gdist * raw;
    if (v) {
      d_sigma[r * N + i] = dal * dist * ex;
      const float w = al * T;
      if (d_rgb) {
        d_rgb[(r * N + i) * 3 + 0] = w * gr0;
        d_rgb[(r * N + i) * 3 + 1] = w * gr1;
        d_rgb[(r * N + i) * 3 + 2] = w * gr2;
      }
      LG[i] = gdist;
    }
  }
  if (d_rd) {
    grdn = wave_sum(grdn);
    if (l < 3) d_rd[r * 3 + l] = grdn * ((l == 0 ? d0 : (l == 1 ? d1 : d2)) / rdn);
  }
  if (d_t) {
    wave_lds_sync();
    // dist_i = (t_{i+1} - t_i) ||rd||: d t_i = ||rd|| (g_{i-1} - g_i), the last dist is constant 0
    for (int i = l; i < N; i += 64) {
      const float gi = (i < N - 1) ? LG[i] : 0.f;
      const float gp = (i > 0) ? LG[i - 1] : 0.f;
      d_t[r * N + i] = rdn * (gp - gi);
    }
  }
}

// ---- cumprod_exclusive (nerf_utils.py:20-25) on n rows of N: out_0 = 1, out_k = prod_{j<k} x_j ------
// One wave per row, chunks of 64, the product carried in fp64 (ATen's CPU cumprod of float accumulates
// in double; the last input is not used, :23).  Backward: d x_i = out_i S_i with
// S_i = sum_{k>i} g_k prod_{i<j<k} x_j (the reverse affine scan suffix_affine, lane map s -> x s + g;
// no division, so exact zeros in x need no special case), d x_{N-1} = 0.
__global__ void __launch_bounds__(256) cumprod_excl_kernel(const float* __restrict__ x, long long n, int N,
                                                           float* __restrict__ out) {
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  double carry = 1.0;
  for (int c = 0; c < N; c += 64) {
    const int i = c + l;
    const float xi = x[r * N + min(i, N - 1)];
    const double inc = wave_incl_prod_d(i < N - 1 ? (double)xi : 1.0);
    const double exc = dpp_fill<0x138>(inc, 1.0);   // wave_shr:1, lane 0 takes 1
    if (i < N) out[r * N + i] = (float)(carry * exc);
    carry = carry * readlane(inc, 63);
  }
}

__global__ void __launch_bounds__(256) cumprod_excl_bwd_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ g, long long n, int N,
                                                               float* __restrict__ dx) {
  __shared__ float lds[4 * COMP_NMAX];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  float* LO = lds + wv * COMP_NMAX;   // the forward's outputs
  double carry = 1.0;
  for (int c = 0; c < N; c += 64) {
    const int i = c + l;
    const float xi = x[r * N + min(i, N - 1)];
    const double inc = wave_incl_prod_d(i < N - 1 ? (double)xi : 1.0);
    const double exc = dpp_fill<0x138>(inc, 1.0);
    if (i < N) LO[i] = (float)(carry * exc);
    carry = carry * readlane(inc, 63);
  }
  wave_lds_sync();
  float cB = 0.f;
  for (int ch = (N + 63) / 64 - 1; ch >= 0; --ch) {
    const int i = ch * 64 + l;
    const bool v = i < N;
    const int ic = min(i, N - 1);
    const float xi = x[r * N + ic], gi = g[r * N + ic];
    const float Sk = suffix_affine(v ? xi : 1.f, v ? gi : 0.f, cB);
    if (v) dx[r * N + i] = (i < N - 1) ? LO[ic] * Sk : 0.f;
  }
}

// ---- compute_query_points_from_rays (nerf_utils.py:96-122) --------------------------------------
// rays ro, rd [n][3], near, far [n] -> depth [n][S] = lerp(near, far, i/S) (+ u (far - near)/S when
// randomized: u [n][S] given, or the Philox stream of the fused render's coarse draws), points
// [n][S][3] = ro + rd t, in ATen's rounding order.  Backward to the rays (depth values carry no
// gradient: near / far come from compute_near_far_planes under no_grad, run.py:197-200):
// d ro = sum_i g_i, d rd = sum_i g_i t_i, one wave per ray (fixed-order sums).
__global__ void __launch_bounds__(256) query_points_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                                           const float* __restrict__ nearp,
                                                           const float* __restrict__ farp, long long n, int S,
                                                           int randomize, const float* __restrict__ u,
                                                           unsigned long long seed, unsigned long long offset,
                                                           float* __restrict__ pts, float* __restrict__ depth) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= n * S) return;
  const long long r = k / S;
  const int i = (int)(k - r * S);
  const float nr = nearp[r], fr = farp[r];
  float t = tlerp(nr, fr, fdiv((float)i, (float)S));
  if (randomize) {
    const float uu = u ? u[k] : rng_uniform(seed, offset, r, i, 0);
    t = fadd(t, fmul(uu, fdiv(fsub(fr, nr), (float)S)));
  }
  depth[k] = t;
#pragma unroll
  for (int c = 0; c < 3; ++c) pts[k * 3 + c] = fadd(ro[r * 3 + c], fmul(rd[r * 3 + c], t));
}

__global__ void __launch_bounds__(256) query_points_bwd_kernel(const float* __restrict__ depth,
                                                               const float* __restrict__ g_pts, long long n, int S,
                                                               float* __restrict__ d_ro, float* __restrict__ d_rd) {
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long r = (long long)blockIdx.x * 4 + wv;
  if (r >= n) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
  for (int i = l; i < S; i += 64) {
    const float t = depth[r * S + i];
    const float* g = g_pts + (r * S + i) * 3;
    a0 += g[0];
    a1 += g[1];
    a2 += g[2];
    b0 = fmaf(g[0], t, b0);
    b1 = fmaf(g[1], t, b1);
    b2 = fmaf(g[2], t, b2);
  }
  a0 = wave_sum(a0), a1 = wave_sum(a1), a2 = wave_sum(a2);
  b0 = wave_sum(b0), b1 = wave_sum(b1), b2 = wave_sum(b2);
  if (l < 3) {
    if (d_ro) d_ro[r * 3 + l] = l == 0 ? a0 : (l == 1 ? a1 : a2);
    if (d_rd) d_rd[r * 3 + l] = l == 0 ? b0 : (l == 1 ? b1 : b2);
  }
}

// ---- sampler closure (generator.py:587-681) at caller points -------------------------------
// x [B][P][3] world coordinates -> sigma [B*P], rgb [B*P][3], decoder outputs y [B*P][11]
// (distance + 10 logits / colour features; optional).  One wave per 64 points of one image.
struct SamplerArgs {
  nfi_field f;
  const float* x;
  int B;
  long long P;
  float* sigma;
  float* rgb;
  float* y;
  // backward
  const float* g_sigma;   // [B*P] or NULL
  const float* g_rgb;     // [B*P][3] or NULL
  const float* g_y;       // [B*P][11] or NULL (dL/d decoder outputs from the caller's own maps)
  float* d_planes;        // field.planes' layout, accumulated (float atomics); NULL: not needed
  float* d_palette_part;  // [B * chunks][30] per-chunk partial, or NULL
  float* d_x;             // [B*P][3] or NULL
};

__device__ __forceinline__ void sampler_point(const SamplerArgs& A, long long gp, PointP& P) {
  const float sr = A.f.scene_range;
#pragma unroll
  for (int k = 0; k < 3; ++k) P.cx[k] = fdiv(A.x[gp * 3 + k], sr);   // x_in / scene_range (generator.py:604)
  P.mask = (fabsf(P.cx[0]) > 1.f || fabsf(P.cx[1]) > 1.f || fabsf(P.cx[2]) > 1.f) ? 1.f : 0.f;
  plane_params(P.cx[0], P.cx[1], A.f.R, P.pl[0]);
  plane_params(P.cx[0], P.cx[2], A.f.R, P.pl[1]);
  plane_params(P.cx[1], P.cx[2], A.f.R, P.pl[2]);
}

__global__ void __launch_bounds__(256) sampler_fwd_kernel(SamplerArgs A) {
  __shared__ __attribute__((aligned(16))) float lds[4 * XTILE];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long cpi = (A.P + 63) / 64;
  const long long job = (long long)blockIdx.x * 4 + wv;
  if (job >= (long long)A.B * cpi) return;
  const int b = (int)(job / cpi);
  const long long p0 = (job % cpi) * 64;
  const int npts = (int)min(64LL, A.P - p0);
  const long long gp = (long long)b * A.P + p0 + min(l, npts - 1);
  float* X = lds + wv * XTILE;
  PointP P;
  sampler_point(A, gp, P);
  const PlaneView pv{A.f.planes + (long long)b * A.f.sb, (int)A.f.sq, (int)A.f.st, A.f.R};
  gather_features(pv, P, npts, X);
  wave_lds_sync();
  float y[NO];
  mlp_forward<NO, true>(A.f.dec, X, npts, y);
  Head h;
  head_forward(y, P.mask, A.f.inv_alpha, A.f.beta, A.f.palette ? A.f.palette + b * (NA * 3) : nullptr, A.f.heads, h);
  if (l < npts) {
    A.sigma[gp] = h.sigma;
#pragma unroll
    for (int c = 0; c < 3; ++c) A.rgb[gp * 3 + c] = h.rgb[c];
    if (A.y) {
#pragma unroll
      for (int k = 0; k < NO; ++k) A.y[gp * NO + k] = y[k];
    }
  }
}

// Backward: re-gather + decoder forward, head backward (+ the caller's dL/dy), decoder input
// gradient on the matrix cores, then per point and plane the bilinear tap's adjoint: d planes by
// float atomics (two 256-B wave instructions per plane: texels x0, x0+1 x 32 channels of rows y0,
// y1) and the grid gradient (ATen grid_sampler_2d border / align_corners rule) -> d x.
__global__ void __launch_bounds__(256) sampler_bwd_kernel(SamplerArgs A) {
  __shared__ __attribute__((aligned(16))) float lds[4 * XTILE];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long cpi = (A.P + 63) / 64;
  const long long job = (long long)blockIdx.x * 4 + wv;
  if (job >= (long long)A.B * cpi) return;
  const int b = (int)(job / cpi);
  const long long p0 = (job % cpi) * 64;
  const int npts = (int)min(64LL, A.P - p0);
  const bool v = l < npts;
  const long long gp = (long long)b * A.P + p0 + min(l, npts - 1);
  float* X = lds + wv * XTILE;
  PointP P;
  sampler_point(A, gp, P);
  const PlaneView pv{A.f.planes + (long long)b * A.f.sb, (int)A.f.sq, (int)A.f.st, A.f.R};
  gather_features(pv, P, npts, X);
  wave_lds_sync();
  // decoder inputs in the MFMA operand layout (lane (j, q): channels 8q.. of point 16sb + j)
  f4v xa[4], xb[4];
  {
    const int j = l & 15, q = l >> 4;
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const bool vp = 16 * sb + j < npts;
      const f4v z{0.f, 0.f, 0.f, 0.f};
      const f4v a0 = ld4(X + (16 * sb + j) * XS + 8 * q), a1 = ld4(X + (16 * sb + j) * XS + 8 * q + 4);
      xa[sb] = vp ? a0 : z;
      xb[sb] = vp ? a1 : z;
    }
  }
  float y[NO];
  mlp_forward<NO, true>(A.f.dec, X, npts, y);
  const float* pal = A.f.palette ? A.f.palette + b * (NA * 3) : nullptr;
  Head h;
  head_forward(y, P.mask, A.f.inv_alpha, A.f.beta, pal, A.f.heads, h);
  float gy[NO];
#pragma unroll
  for (int k = 0; k < NO; ++k) gy[k] = (A.g_y && v) ? A.g_y[gp * NO + k] : 0.f;
  const float gs = (A.g_sigma && v) ? A.g_sigma[gp] : 0.f;
  if (A.f.heads & NFI_HEAD_NERF_DENSITY) {
    const float z = fsub(y[0], 1.f);
    const float gm = fmul(gs, fsub(1.f, P.mask));
    const float ez = expf(z);
    gy[0] += z > 20.f ? gm : gm * (ez / (ez + 1.f));
  } else {
    const float xn = -y[0];
    const float sgn = tsign(xn);
    const float ex2 = expf(-fabsf(xn) / A.f.beta);
    const float gcdf = (gs * A.f.inv_alpha) * (1.f - P.mask);
    gy[0] += -(((gcdf * 0.5f * sgn) * ex2 / A.f.beta) * sgn);
  }
  float gc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) gc[c] = (A.g_rgb && v) ? A.g_rgb[gp * 3 + c] : 0.f;
  wave_lds_sync();
  if (A.f.heads & NFI_HEAD_RGB_SIGMOID) {
#pragma unroll
    for (int c = 0; c < 3; ++c) gy[1 + c] += fmul(fmul(gc[c], 2.004f), fsub(1.f, h.p[c])) * h.p[c];
  } else {
    float gp_[NA], dot = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      gp_[k] = gc[0] * pal[k * 3 + 0] + gc[1] * pal[k * 3 + 1] + gc[2] * pal[k * 3 + 2];
      dot = fmaf(gp_[k], h.p[k], dot);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) gy[1 + k] += (gp_[k] - dot) * h.p[k];
    float pv[NA * 3];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      pv[k * 3 + 0] = h.p[k] * gc[0];
      pv[k * 3 + 1] = h.p[k] * gc[1];
      pv[k * 3 + 2] = h.p[k] * gc[2];
    }
    lds_store_keep(X + l * XS, pv);
    wave_lds_sync();
    if (A.d_palette_part) {
      const int col = l & 31, r0 = (l >> 5) * 32;
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      if (col < NA * 3) {
#pragma unroll
        for (int jj = 0; jj < 32; ++jj) s4[jj & 3] += X[(r0 + jj) * XS + col];
      }
      const float sh = sum_halves((s4[0] + s4[1]) + (s4[2] + s4[3]));
      if (l < NA * 3) A.d_palette_part[job * (NA * 3) + l] = sh;
    }
  }
  // dY^T operands through the tile
  wave_lds_sync();
  {
    float dyr[DYC<NO>];
#pragma unroll
    for (int o = 0; o < DYC<NO>; ++o) dyr[o] = (o < NO && v) ? gy[o] : 0.f;
    lds_store_keep(X + l * XS, dyr);
  }
  wave_lds_sync();
  f4v gxo[2][4];
  mlp_backward<NO>(A.f.dec, xa, xb, X, 1.f / 3.f, [&](int cb, int sb, f4v gv) { gxo[cb][sb] = gv; });
  // each plane's tap feature gradient dX/3 into the tile: row = point, 32 channels
  wave_lds_sync();
  {
    const int j = l & 15, q = l >> 4;
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        *reinterpret_cast<f4v*>(X + (16 * sb + j) * XS + 16 * cb + 4 * q) = gxo[cb][sb];
  }
  wave_lds_sync();
  // adjoint of the three bilinear taps, point by point: lane (dx = l >> 5, c = l & 31)
  const int dx = l >> 5, c = l & 31;
  float* dpl = A.d_planes ? A.d_planes + (long long)b * A.f.sb : nullptr;
  float gxs = 0.f, gys = 0.f, gzs = 0.f;   // this lane's point's d x (normalised coordinates)
  for (int jp = 0; jp < npts; ++jp) {
    const float g = X[jp * XS + c];
    float du[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int pk = __shfl(P.pl[q].tex, jp);
      const float w = __shfl(P.pl[q].w, jp), nn = __shfl(P.pl[q].n, jp);
      const float e = 1.f - w, s = 1.f - nn;
      const int t0 = (pk & 0xFFFFF) + (dx ? ((pk >> 20) & 1) : 0);
      const int t1 = t0 + (((pk >> 21) & 1) ? pv.R : 0);
      const float wx = dx ? w : e;
      if (dpl) {
        atomicAdd(dpl + q * pv.sq + (long long)t0 * pv.st + c, g * (s * wx));
        atomicAdd(dpl + q * pv.sq + (long long)t1 * pv.st + c, g * (nn * wx));
      }
      if (A.d_x) {
        const float v0 = pv.base[q * pv.sq + (long long)t0 * pv.st + c];
        const float v1 = pv.base[q * pv.sq + (long long)t1 * pv.st + c];
        // d feat / d ix = s (V(x1,y0) - V(x0,y0)) + n (V(x1,y1) - V(x0,y1)); d / d iy = e (V(x0,y1) -
        // V(x0,y0)) + w (V(x1,y1) - V(x1,y0))
        const float gix = wave_sum(g * ((dx ? 1.f : -1.f) * (s * v0 + nn * v1)));
        const float giy = wave_sum(g * (wx * (v1 - v0)));
        const float gxm = __shfl(P.pl[q].gxm, jp), gym = __shfl(P.pl[q].gym, jp);
        du[q == 2 ? 1 : 0] += gix * gxm;          // xy, xz: u = x0; yz: u = x1
        du[q == 0 ? 1 : 2] += giy * gym;          // xy: v = x1; xz, yz: v = x2
      }
    }
    if (l == jp) {
      gxs = du[0];
      gys = du[1];
      gzs = du[2];
    }
  }
  if (A.d_x && v) {
    const float sr = A.f.scene_range;
    A.d_x[gp * 3 + 0] = fdiv(gxs, sr);
    A.d_x[gp * 3 + 1] = fdiv(gys, sr);
    A.d_x[gp * 3 + 2] = fdiv(gzs, sr);
  }
}

struct Workspace {
  float* gfeat;
  float* gsig;
  float* wts;
  int* counts;
  int* cursor;
  int* offsets;
  int* chunk_start;
  int* chunk_tile;
  int* meta;
  int* part;
  int4* list;
  float* dpc;
  int* check;        // -DNFI_TILE_CHECK builds: counters + first failure + two double sums
  float* shadow;     // -DNFI_TILE_CHECK builds: the second d-planes sum and a snapshot of d planes
  float* snapshot;
  // deterministic mode
  int4* det_list;    // the entries in tile, sample order (+ 64 zeroed records)
  float* tpart;      // per-chunk partial tile images
  long long bytes;
};

// deterministic mode of the backward, per host thread (nfi_set_deterministic; default from the
// environment variable NFI_DETERMINISTIC)
static thread_local int g_det = -1;
static bool deterministic() {
  if (g_det < 0) {
    const char* e = std::getenv("NFI_DETERMINISTIC");
    g_det = (e && e[0] && std::strcmp(e, "0") != 0) ? 1 : 0;
  }
  return g_det != 0;
}

static Workspace carve(const nfi_render_args* a, void* base) {
  const long long nrays = (long long)a->B * a->HW;
  const int N = a->fine ? 2 * a->S : a->S;
  const long long nsamp = nrays * N;
  const TileGrid tg = tile_grid(a->field.R, a->HW, a->W, N);
  const long long K = (long long)a->B * beams_per_image(tg) * 3 * tg.nx * tg.ny;
  char* p = static_cast<char*>(base);
  Workspace w;
  auto take = [&](long long bytes) {
    char* q = p;
    p += (bytes + 255) / 256 * 256;
    return q;
  };
  w.gfeat = reinterpret_cast<float*>(take(nsamp * NC * 4));
  w.gsig = reinterpret_cast<float*>(take(nsamp * 4));
  w.wts = reinterpret_cast<float*>(take(nsamp * 4));
  w.counts = reinterpret_cast<int*>(take(K * 4));
  w.cursor = reinterpret_cast<int*>(take(K * 4));
  w.offsets = reinterpret_cast<int*>(take((K + 1) * 4));
  w.chunk_start = reinterpret_cast<int*>(take((K + 1) * 4));
  w.meta = reinterpret_cast<int*>(take(16));
  w.part = reinterpret_cast<int*>(take((K / 1024 + 1) * 8));
  // chunks <= ceil(entries / CHUNK) + K  (each tile wastes at most one partial chunk)
  w.chunk_tile = reinterpret_cast<int*>(take((3 * nsamp / CHUNK + K + 1) * 4));
  w.list = reinterpret_cast<int4*>(take((3 * nsamp + 128) * 16));   // + padding read by tile_chunk
  w.dpc = reinterpret_cast<float*>(take(nsamp * 6 * 4));
  w.check = nullptr;
  w.shadow = w.snapshot = nullptr;
  w.det_list = nullptr;
  w.tpart = nullptr;
  if (deterministic()) {
    w.det_list = reinterpret_cast<int4*>(take((3 * nsamp + 128) * 16));
    w.tpart = reinterpret_cast<float*>(take((3 * nsamp / CHUNK + K + 1) * (TTX * TTY * NC) * 4));
  }
#if NFI_TILE_CHECK
  w.check = reinterpret_cast<int*>(take(64 * 4));
  w.shadow = reinterpret_cast<float*>(take((long long)a->B * a->field.sb * 4));
  w.snapshot = reinterpret_cast<float*>(take((long long)a->B * a->field.sb * 4));
#endif
  w.bytes = p - static_cast<char*>(base);
  return w;
}

template <int SPL, int NPL, bool FINE, int NOUT>
static int launch_fwd(const nfi_render_args* a, hipStream_t s) {
  const long long nrays = (long long)a->B * a->HW;
  if (a->tile_counts) {
    const TileGrid tg = tile_grid(a->field.R, a->HW, a->W, FINE ? 2 * a->S : a->S);
    NFI_REQUIRE(hipMemsetAsync(a->tile_counts, 0, (size_t)a->B * beams_per_image(tg) * 3 * tg.nx * tg.ny * 4, s) == hipSuccess,
                "render_forward: memset failed");
  }
  render_fwd_kernel<SPL, NPL, FINE, NOUT><<<(unsigned)((nrays + 3) / 4), 256, 0, s>>>(*a);
  NFI_CHECK_LAUNCH("render_fwd_kernel");
  if (a->extras) {
    const int N = FINE ? 2 * a->S : a->S;
    const unsigned grid = (unsigned)((nrays + 3) / 4);
    constexpr int EN = NOUT;
    if (N <= 64) extras_kernel<1, EN><<<grid, 256, 0, s>>>(*a);
    else if (N <= 128) extras_kernel<2, EN><<<grid, 256, 0, s>>>(*a);
    else extras_kernel<4, EN><<<grid, 256, 0, s>>>(*a);
    NFI_CHECK_LAUNCH("extras_kernel");
  }
  return NFI_OK;
}

static int launch_bwd(const nfi_render_args* a, const nfi_render_grad_args* g, hipStream_t s, int stage) {
  const long long nrays = (long long)a->B * a->HW;
  const int N = a->fine ? 2 * a->S : a->S;
  const long long nsamp = nrays * N;
  const TileGrid tg = tile_grid(a->field.R, a->HW, a->W, N);
  const int K = a->B * beams_per_image(tg) * 3 * tg.nx * tg.ny;
  Workspace w = carve(a, g->workspace);
  NFI_REQUIRE(w.bytes <= g->workspace_bytes, "render_backward: workspace too small (%lld < %lld)",
              (long long)g->workspace_bytes, w.bytes);
  NFI_REQUIRE(nsamp * 3 < (1LL << 31), "render_backward: too many samples per call (%lld)", nsamp);
  // 1) bin (sample, plane) entries by plane tile from the saved depths.  With the forward's
  //    tile counts only the scan runs here and field_bwd fills the bins (its atomics hide
  //    behind the MLP); otherwise count here and fill in bin_fill_kernel.
  const bool do_bins = stage < 0 || stage == 0, do_field = stage < 0 || stage == 1, do_tiles = stage < 0 || stage == 2;
  const bool fwd_counts = g->tile_counts != nullptr;
  const int* counts = fwd_counts ? g->tile_counts : w.counts;
  BinArgs B{a->ro, a->rd, a->t_saved, nsamp, N, a->HW, a->field.R, tg, a->field.scene_range,
            w.counts, w.cursor, w.list};
  const unsigned sb = (unsigned)((nsamp + 255) / 256);
  if (do_bins) {
    if (!fwd_counts) {
      NFI_REQUIRE(hipMemsetAsync(w.counts, 0, (size_t)K * 4, s) == hipSuccess, "render_backward: memset failed");
      bin_count_kernel<<<sb, 256, 0, s>>>(B);
      NFI_CHECK_LAUNCH("bin_count_kernel");
    }
    const unsigned nb = (unsigned)((K + 1023) / 1024);
    scan_partials_kernel<<<nb, 1024, 0, s>>>(counts, K, w.part);
    NFI_CHECK_LAUNCH("scan_partials_kernel");
    scan_blocks_kernel<<<nb, 1024, 0, s>>>(counts, K, w.part, w.offsets, w.cursor, w.chunk_start, w.meta);
    NFI_CHECK_LAUNCH("scan_blocks_kernel");
    chunk_map_kernel<<<(unsigned)((K + 255) / 256), 256, 0, s>>>(counts, w.chunk_start, K, w.chunk_tile, w.offsets,
                                                               w.list);
    NFI_CHECK_LAUNCH("chunk_map_kernel");
    if (!fwd_counts) {
      bin_fill_kernel<<<sb, 256, 0, s>>>(B);
      NFI_CHECK_LAUNCH("bin_fill_kernel");
    }
  }
  // 2) per-ray compositing backward, then per-(ray, 64-sample chunk) field backward
  const int NPL = (N + 63) / 64;
  BwdArgs bg{g->g_rgb, g->g_mask, g->d_palette_ray, g->g_ro, g->g_rd, w.gfeat, w.gsig, w.wts, NPL,
             fwd_counts ? w.cursor : nullptr, w.list, tg, g->d_xray};
  const unsigned rb = (unsigned)((nrays + 3) / 4);
  if (do_field) {
    if (NPL <= 1) composite_bwd_kernel<1><<<rb, 256, 0, s>>>(*a, bg);
    else if (NPL <= 2) composite_bwd_kernel<2><<<rb, 256, 0, s>>>(*a, bg);
    else composite_bwd_kernel<4><<<rb, 256, 0, s>>>(*a, bg);
    NFI_CHECK_LAUNCH("composite_bwd_kernel");
    if (a->field.heads & NFI_HEAD_VIEWDIR)
      field_bwd_kernel<true, NOV><<<(unsigned)((nrays * NPL + 3) / 4), 256, 0, s>>>(*a, bg);
    else if (a->field.heads)
      field_bwd_kernel<true, NO><<<(unsigned)((nrays * NPL + 3) / 4), 256, 0, s>>>(*a, bg);
    else
      field_bwd_kernel<false, NO><<<(unsigned)((nrays * NPL + 3) / 4), 256, 0, s>>>(*a, bg);
    NFI_CHECK_LAUNCH("field_bwd_kernel");
  }
#if defined(NFI_ABLATE) && NFI_ABLATE == 5
  float* const dpc_used = nullptr;   // experiment: no pose path in the tile pass
#else
  float* const dpc_used = g->g_ro ? w.dpc : nullptr;
#endif
  const bool det = w.tpart != nullptr;
  TileArgs TA{a->field.planes, dpc_used, w.gfeat, counts, w.offsets, w.chunk_start,
              w.chunk_tile, w.meta, det ? w.det_list : w.list, g->d_planes, a->field.sb, (int)a->field.sq,
              (int)a->field.st, a->field.R, tg, w.cursor, w.check, w.shadow, nsamp, K, w.tpart};
  if (do_tiles) {
    // 3) per-tile register accumulation of d planes (+ per-entry grid gradients for the pose)
    // (a bound on the chunk count meta[0]; the chunk queue meta[1] starts at 0)
    const long long TB = 3 * nsamp / CHUNK + K + 1;
    NFI_REQUIRE(hipMemsetAsync(w.meta + 1, 0, 4, s) == hipSuccess, "render_backward: memset failed");
#if NFI_TILE_CHECK
    const size_t dpb = (size_t)a->B * a->field.sb * 4;
    NFI_REQUIRE(hipMemsetAsync(w.check, 0, 64 * 4, s) == hipSuccess && hipMemsetAsync(w.shadow, 0, dpb, s) == hipSuccess &&
                    hipMemcpyAsync(w.snapshot, g->d_planes, dpb, hipMemcpyDeviceToDevice, s) == hipSuccess,
                "render_backward: check-build setup failed");
#endif
    if (det) {
      // the bins' entries in sample order per tile (their append order follows the cursor atomics)
      det_sort_kernel<<<(unsigned)(3 * nsamp / CHUNK + K + 1), 256, 0, s>>>(w.list, w.offsets, w.chunk_start,
                                                                             w.chunk_tile, w.meta, w.det_list);
      NFI_CHECK_LAUNCH("det_sort_kernel");
      det_pad_kernel<<<1, 64, 0, s>>>(w.offsets, K, w.det_list);
      NFI_CHECK_LAUNCH("det_pad_kernel");
    }
    tile_kernel<<<(unsigned)std::min<long long>(TB, TILE_WGS), 256, 0, s>>>(TA);
    NFI_CHECK_LAUNCH("tile_kernel");
    if (det) {
      const long long n = (long long)a->B * 3 * a->field.R * a->field.R * NC;
      dplanes_reduce_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(w.tpart, w.chunk_start, tg, a->B, a->field.R,
                                                                         a->field.sb, (int)a->field.sq,
                                                                         (int)a->field.st, g->d_planes);
      NFI_CHECK_LAUNCH("dplanes_reduce_kernel");
    }
#if NFI_TILE_CHECK
    {
      const long long ne = (long long)a->B * a->field.sb;
      tile_shadow_compare_kernel<<<(unsigned)std::min<long long>((ne + 255) / 256, 4096), 256, 0, s>>>(
          g->d_planes, w.snapshot, w.shadow, ne, reinterpret_cast<double*>(w.check + 40));
      NFI_CHECK_LAUNCH("tile_shadow_compare_kernel");
      int hc[64];
      NFI_REQUIRE(hipMemcpyAsync(hc, w.check, sizeof(hc), hipMemcpyDeviceToHost, s) == hipSuccess &&
                      hipStreamSynchronize(s) == hipSuccess,
                  "render_backward: check readback failed");
      double sums[2];
      memcpy(sums, hc + 40, sizeof(sums));
      const double rel = sums[1] > 0 ? sqrt(sums[0] / sums[1]) : sqrt(sums[0]);
      int nbad = 0;
      for (int k = 1; k < 31; ++k) nbad += hc[k];
      if (nbad || !(rel <= 1e-5)) {
        set_error("tile check: %d violations (first: code %d chunk %d tile %d lane %d value %d expected %d; "
                  "per code 1..12: %d %d %d %d %d %d %d %d %d %d %d %d); d planes vs the per-entry sum: "
                  "rel L2 %.3g",
                  nbad, hc[32], hc[33], hc[34], hc[35], hc[36], hc[37], hc[1], hc[2], hc[3], hc[4], hc[5], hc[6],
                  hc[7], hc[8], hc[9], hc[10], hc[11], hc[12], rel);
        return NFI_ECHECK;
      }
    }
#endif
    // 4) ray-coordinate gradients
#if defined(NFI_ABLATE) && (NFI_ABLATE == 5 || NFI_ABLATE == 6)
    if (false) {   // experiment: no reduce launch
#else
    if (g->g_ro) {
#endif
      if (NPL <= 1) dcoord_reduce_kernel<1><<<rb, 256, 0, s>>>(*a, bg, w.dpc);
      else if (NPL <= 2) dcoord_reduce_kernel<2><<<rb, 256, 0, s>>>(*a, bg, w.dpc);
      else dcoord_reduce_kernel<4><<<rb, 256, 0, s>>>(*a, bg, w.dpc);
      NFI_CHECK_LAUNCH("dcoord_reduce_kernel");
    }
  }
  return NFI_OK;
}

template <int NOUT>
static int dispatch_fwd_n(const nfi_render_args* a, hipStream_t s) {
  const int S = a->S;
  if (a->fine) {
    if (S >= 3 && S <= 32) return launch_fwd<1, 1, true, NOUT>(a, s);
    if (S >= 3 && S <= 64) return launch_fwd<1, 2, true, NOUT>(a, s);
    if (S >= 3 && S <= 128) return launch_fwd<2, 4, true, NOUT>(a, s);
  } else {
    if (S >= 1 && S <= 64) return launch_fwd<1, 1, false, NOUT>(a, s);
    if (S >= 1 && S <= 128) return launch_fwd<2, 2, false, NOUT>(a, s);
    if (S >= 1 && S <= 256) return launch_fwd<4, 4, false, NOUT>(a, s);
  }
  return NFI_EINVAL;
}

static int dispatch_fwd(const nfi_render_args* a, hipStream_t s) {
  const int S = a->S;
  const int e = (a->field.heads & NFI_HEAD_VIEWDIR) ? dispatch_fwd_n<NOV>(a, s) : dispatch_fwd_n<NO>(a, s);
  if (e != NFI_EINVAL) return e;
  set_error("render: unsupported samples per ray S=%d (fine=%d): need 3..128 with fine sampling, "
            "1..256 without", S, (int)a->fine);
  return NFI_EINVAL;
}

static bool supported_S(const nfi_render_args* a) {
  return a->fine ? (a->S >= 3 && a->S <= 128) : (a->S >= 1 && a->S <= 256);
}

static int validate(const nfi_render_args* a) {
  NFI_REQUIRE(a != nullptr, "render: null args");
  const nfi_field& f = a->field;
  NFI_REQUIRE((f.heads & ~(NFI_HEAD_RGB_SIGMOID | NFI_HEAD_NERF_DENSITY | NFI_HEAD_VIEWDIR)) == 0,
              "render: unknown heads bits 0x%x", f.heads);
  NFI_REQUIRE(!(f.heads & NFI_HEAD_VIEWDIR) ||
                  (f.xray && f.vhead && f.vhead_out == ((f.heads & NFI_HEAD_RGB_SIGMOID) ? 3 : NA)),
              "render: NFI_HEAD_VIEWDIR needs xray, vhead and vhead_out = %d (got %d)",
              (f.heads & NFI_HEAD_RGB_SIGMOID) ? 3 : NA, f.vhead_out);
  NFI_REQUIRE(f.planes && f.dec && (f.palette || (f.heads & NFI_HEAD_RGB_SIGMOID)), "render: null field pointer");
  NFI_REQUIRE(f.R >= 2 && f.R <= 1024, "render: plane resolution R=%d out of range [2,1024]", f.R);
  NFI_REQUIRE(f.st >= NC && 3LL * f.sq < (1LL << 31) && (long long)f.R * f.R * f.st < (1LL << 31),
              "render: plane strides out of range (st=%lld sq=%lld)", (long long)f.st, (long long)f.sq);
  NFI_REQUIRE(((f.heads & NFI_HEAD_NERF_DENSITY) || (f.beta > 0.f && std::isfinite(f.inv_alpha))) &&
                  f.scene_range > 0.f, "render: bad field scalars");
  NFI_REQUIRE(a->ro && a->rd && a->near_ && a->far_, "render: null ray pointer");
  NFI_REQUIRE(a->B > 0 && a->HW > 0, "render: bad shape B=%d HW=%d", a->B, a->HW);
  {
    const bool all = a->t_saved && a->sigma_saved && a->rgb_saved && a->y_saved && a->perm;
    const bool none = !a->t_saved && !a->sigma_saved && !a->rgb_saved && !a->y_saved && !a->perm;
    NFI_REQUIRE(all || none, "render: saved-state pointers must be all set or all null");
  }
  NFI_REQUIRE(supported_S(a), "render: unsupported samples per ray S=%d (fine=%d): need 3..128 with fine "
              "sampling, 1..256 without", a->S, (int)a->fine);
  return NFI_OK;
}

}  // namespace nfi

extern "C" {

int32_t nfi_render_forward(const nfi_render_args* a, void* stream) {
  int e = nfi::validate(a);
  if (e) return e;
  NFI_REQUIRE(a->rgb && a->depth && a->mask, "render_forward: null output");
  NFI_REQUIRE(a->t_saved || (!a->extras && !a->tile_counts && !a->x_saved),
              "render_forward: eval outputs / backward state need the saved-state buffers");
  NFI_REQUIRE((a->extras & ~7) == 0, "render_forward: unknown extras bits 0x%x", a->extras);
  NFI_REQUIRE(!(a->extras & 1) || (a->normal_map && a->x_saved),
              "render_forward: normals need normal_map and x_saved");
  NFI_REQUIRE(!(a->extras & 6) || a->semantic_map, "render_forward: semantics/coords need semantic_map");
  NFI_REQUIRE(!(a->extras & 1) || !(a->field.heads & NFI_HEAD_NERF_DENSITY),
              "render_forward: normals need the SDF field (run.py:229)");
  NFI_REQUIRE((a->extras & 6) != 2 || !(a->field.heads & NFI_HEAD_RGB_SIGMOID),
              "render_forward: semantics need attention values (run.py:232)");
  return nfi::dispatch_fwd(a, (hipStream_t)stream);
}

int64_t nfi_tile_count_size(const nfi_render_args* a) {
  if (nfi::validate(a)) return -1;
  const nfi::TileGrid tg = nfi::tile_grid(a->field.R, a->HW, a->W, a->fine ? 2 * a->S : a->S);
  return (int64_t)a->B * nfi::beams_per_image(tg) * 3 * tg.nx * tg.ny;
}

int64_t nfi_tile_count_size_shape(int32_t B, int32_t R, int32_t H, int32_t W, int32_t N) {
  if (B <= 0 || R < 2 || H <= 0 || W <= 0 || N <= 0) return -1;
  const nfi::TileGrid tg = nfi::tile_grid(R, H * W, W, N);
  return (int64_t)B * nfi::beams_per_image(tg) * 3 * tg.nx * tg.ny;
}

int32_t nfi_set_deterministic(int32_t on) {
  const int32_t prev = nfi::deterministic() ? 1 : 0;
  if (on >= 0) nfi::g_det = on ? 1 : 0;
  return prev;
}

int64_t nfi_render_backward_workspace_bytes(const nfi_render_args* a) {
  if (nfi::validate(a)) return -1;
  return nfi::carve(a, nullptr).bytes;
}

int32_t nfi_render_backward(const nfi_render_args* a, const nfi_render_grad_args* g, void* stream) {
  int e = nfi::validate(a);
  if (e) return e;
  NFI_REQUIRE(g && g->g_rgb && g->g_mask && g->d_planes && g->workspace &&
                  (g->d_palette_ray || (a->field.heads & NFI_HEAD_RGB_SIGMOID)),
              "render_backward: null grad pointer");
  NFI_REQUIRE(a->x_saved && a->t_saved,
              "render_backward: the forward's saved state (x_saved, t/sigma/rgb/y/perm) is required");
  NFI_REQUIRE((g->g_ro == nullptr) == (g->g_rd == nullptr), "render_backward: g_ro/g_rd must both be set or null");
  NFI_REQUIRE(!(a->field.heads & NFI_HEAD_VIEWDIR) || g->d_xray, "render_backward: NFI_HEAD_VIEWDIR needs d_xray");
  return nfi::launch_bwd(a, g, (hipStream_t)stream, -1);
}

int32_t nfi_render_backward_stage(const nfi_render_args* a, const nfi_render_grad_args* g, int32_t stage,
                                  void* stream) {
  int e = nfi::validate(a);
  if (e) return e;
  NFI_REQUIRE(g && g->g_rgb && g->g_mask && g->d_planes && g->workspace &&
                  (g->d_palette_ray || (a->field.heads & NFI_HEAD_RGB_SIGMOID)),
              "render_backward: null grad pointer");
  NFI_REQUIRE(a->x_saved && a->t_saved,
              "render_backward: the forward's saved state (x_saved, t/sigma/rgb/y/perm) is required");
  NFI_REQUIRE((g->g_ro == nullptr) == (g->g_rd == nullptr), "render_backward: g_ro/g_rd must both be set or null");
  NFI_REQUIRE(stage >= 0 && stage <= 2, "render_backward_stage: stage %d not in 0..2", stage);
  NFI_REQUIRE(!(a->field.heads & NFI_HEAD_VIEWDIR) || g->d_xray, "render_backward: NFI_HEAD_VIEWDIR needs d_xray");
  return nfi::launch_bwd(a, g, (hipStream_t)stream, stage);
}

// ---- per-stage seams ----

int32_t nfi_sample_pdf(const float* bins, const float* weights, int64_t n, int32_t nbins, int32_t num_samples,
                       int32_t deterministic, const float* u, uint64_t seed, uint64_t offset, float* out,
                       void* stream) {
  NFI_REQUIRE(bins && weights && out, "sample_pdf: null pointer");
  NFI_REQUIRE(n > 0 && nbins >= 2 && nbins <= nfi::PDF_NBMAX && num_samples > 0,
              "sample_pdf: bad shape n=%lld nbins=%d (2..%d) num_samples=%d", (long long)n, nbins, nfi::PDF_NBMAX,
              num_samples);
  nfi::sample_pdf_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      bins, weights, n, nbins, num_samples, deterministic, u, seed, offset, out);
  NFI_CHECK_LAUNCH("sample_pdf_kernel");
  return NFI_OK;
}

int32_t nfi_composite_forward(const float* sigma, const float* rgb, const float* rd, const float* t, int64_t n,
                              int32_t N, int32_t white_bg, float* rgb_map, float* depth, float* mask, float* weights,
                              void* stream) {
  NFI_REQUIRE(sigma && rgb && rd && t && rgb_map && depth && mask, "composite_forward: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1 && N <= nfi::COMP_NMAX, "composite_forward: bad shape n=%lld N=%d (1..%d)",
              (long long)n, N, nfi::COMP_NMAX);
  nfi::composite_fwd_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      sigma, rgb, rd, t, n, N, white_bg, rgb_map, depth, mask, weights);
  NFI_CHECK_LAUNCH("composite_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_composite_backward(const float* sigma, const float* rgb, const float* rd, const float* t, int64_t n,
                               int32_t N, int32_t white_bg, const float* g_rgb, const float* g_mask,
                               const float* g_weights, float* d_sigma, float* d_rgb, float* d_rd, float* d_t,
                               void* stream) {
  NFI_REQUIRE(sigma && rgb && rd && t && g_rgb && g_mask && d_sigma && d_rgb, "composite_backward: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1 && N <= nfi::COMP_NMAX, "composite_backward: bad shape n=%lld N=%d (1..%d)",
              (long long)n, N, nfi::COMP_NMAX);
  nfi::composite_bwd_seam_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      sigma, rgb, rd, t, n, N, white_bg, g_rgb, g_mask, g_weights, d_sigma, d_rgb, d_rd, d_t);
  NFI_CHECK_LAUNCH("composite_bwd_seam_kernel");
  return NFI_OK;
}

int32_t nfi_volume_weights_forward(const float* sigma, const float* rd, const float* t, int64_t n, int32_t N,
                                   float* weights, void* stream) {
  NFI_REQUIRE(sigma && rd && t && weights, "volume_weights_forward: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1 && N <= nfi::COMP_NMAX, "volume_weights_forward: bad shape n=%lld N=%d (1..%d)",
              (long long)n, N, nfi::COMP_NMAX);
  nfi::composite_fwd_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      sigma, nullptr, rd, t, n, N, 0, nullptr, nullptr, nullptr, weights);
  NFI_CHECK_LAUNCH("composite_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_volume_weights_backward(const float* sigma, const float* rd, const float* t, int64_t n, int32_t N,
                                    const float* g_weights, float* d_sigma, float* d_rd, float* d_t, void* stream) {
  NFI_REQUIRE(sigma && rd && t && g_weights && d_sigma, "volume_weights_backward: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1 && N <= nfi::COMP_NMAX, "volume_weights_backward: bad shape n=%lld N=%d (1..%d)",
              (long long)n, N, nfi::COMP_NMAX);
  nfi::composite_bwd_seam_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      sigma, nullptr, rd, t, n, N, 0, nullptr, nullptr, g_weights, d_sigma, nullptr, d_rd, d_t);
  NFI_CHECK_LAUNCH("composite_bwd_seam_kernel");
  return NFI_OK;
}

int32_t nfi_cumprod_exclusive(const float* x, int64_t n, int32_t N, float* out, void* stream) {
  NFI_REQUIRE(x && out, "cumprod_exclusive: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1, "cumprod_exclusive: bad shape n=%lld N=%d", (long long)n, N);
  nfi::cumprod_excl_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(x, n, N, out);
  NFI_CHECK_LAUNCH("cumprod_excl_kernel");
  return NFI_OK;
}

int32_t nfi_cumprod_exclusive_backward(const float* x, const float* g_out, int64_t n, int32_t N, float* d_x,
                                       void* stream) {
  NFI_REQUIRE(x && g_out && d_x, "cumprod_exclusive_backward: null pointer");
  NFI_REQUIRE(n > 0 && N >= 1 && N <= nfi::COMP_NMAX, "cumprod_exclusive_backward: bad shape n=%lld N=%d (1..%d)",
              (long long)n, N, nfi::COMP_NMAX);
  nfi::cumprod_excl_bwd_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(x, g_out, n, N, d_x);
  NFI_CHECK_LAUNCH("cumprod_excl_bwd_kernel");
  return NFI_OK;
}

int32_t nfi_query_points(const float* ro, const float* rd, const float* near_, const float* far_, int64_t n,
                         int32_t S, int32_t randomize, const float* u, uint64_t seed, uint64_t offset, float* points,
                         float* depth, void* stream) {
  NFI_REQUIRE(ro && rd && near_ && far_ && points && depth, "query_points: null pointer");
  NFI_REQUIRE(n > 0 && S >= 1 && n * (long long)S < (1LL << 40), "query_points: bad shape n=%lld S=%d",
              (long long)n, S);
  const long long k = n * S;
  nfi::query_points_kernel<<<(unsigned)((k + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      ro, rd, near_, far_, n, S, randomize, u, seed, offset, points, depth);
  NFI_CHECK_LAUNCH("query_points_kernel");
  return NFI_OK;
}

int32_t nfi_query_points_backward(const float* depth, const float* g_points, int64_t n, int32_t S, float* d_ro,
                                  float* d_rd, void* stream) {
  NFI_REQUIRE(depth && g_points && (d_ro || d_rd), "query_points_backward: null pointer");
  NFI_REQUIRE(n > 0 && S >= 1, "query_points_backward: bad shape n=%lld S=%d", (long long)n, S);
  nfi::query_points_bwd_kernel<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(depth, g_points, n, S, d_ro,
                                                                                        d_rd);
  NFI_CHECK_LAUNCH("query_points_bwd_kernel");
  return NFI_OK;
}

static int check_sampler_field(const nfi_field* f, int32_t B, int64_t P) {
  NFI_REQUIRE(f && f->planes && f->dec, "sampler: null field pointer");
  NFI_REQUIRE(B > 0 && P > 0, "sampler: bad shape B=%d P=%lld", B, (long long)P);
  NFI_REQUIRE(f->R >= 2, "sampler: plane resolution R=%d < 2", f->R);
  NFI_REQUIRE(!(f->heads & NFI_HEAD_VIEWDIR),
              "sampler: the view-direction mapper closure needs per-ray inputs (render() only)");
  NFI_REQUIRE((f->heads & ~(NFI_HEAD_RGB_SIGMOID | NFI_HEAD_NERF_DENSITY)) == 0, "sampler: unknown heads 0x%x",
              f->heads);
  NFI_REQUIRE(f->palette || (f->heads & NFI_HEAD_RGB_SIGMOID), "sampler: the attention head needs a palette");
  NFI_REQUIRE(((uintptr_t)f->planes & 15) == 0 && f->st % 4 == 0 && f->sq % 4 == 0 && f->sb % 4 == 0,
              "sampler: planes must be 16-byte aligned with strides divisible by 4");
  NFI_REQUIRE(f->scene_range > 0.f, "sampler: bad scene_range");
  return NFI_OK;
}

int64_t nfi_sampler_chunks(int32_t B, int64_t P) {
  if (B <= 0 || P <= 0) return -1;
  return (int64_t)B * ((P + 63) / 64);
}

int32_t nfi_sampler_forward(const nfi_field* f, const float* x, int32_t B, int64_t P, float* sigma, float* rgb,
                            float* y, void* stream) {
  int e = check_sampler_field(f, B, P);
  if (e) return e;
  NFI_REQUIRE(x && sigma && rgb, "sampler_forward: null pointer");
  nfi::SamplerArgs A{};
  A.f = *f;
  A.x = x;
  A.B = B;
  A.P = P;
  A.sigma = sigma;
  A.rgb = rgb;
  A.y = y;
  const long long jobs = nfi_sampler_chunks(B, P);
  nfi::sampler_fwd_kernel<<<(unsigned)((jobs + 3) / 4), 256, 0, (hipStream_t)stream>>>(A);
  NFI_CHECK_LAUNCH("sampler_fwd_kernel");
  return NFI_OK;
}

int32_t nfi_sampler_backward(const nfi_field* f, const float* x, int32_t B, int64_t P, const float* g_sigma,
                             const float* g_rgb, const float* g_y, float* d_planes, float* d_palette_part,
                             float* d_x, void* stream) {
  int e = check_sampler_field(f, B, P);
  if (e) return e;
  NFI_REQUIRE(x, "sampler_backward: null pointer");
  NFI_REQUIRE(d_palette_part || (f->heads & NFI_HEAD_RGB_SIGMOID),
              "sampler_backward: the attention head needs d_palette_part");
  nfi::SamplerArgs A{};
  A.f = *f;
  A.x = x;
  A.B = B;
  A.P = P;
  A.g_sigma = g_sigma;
  A.g_rgb = g_rgb;
  A.g_y = g_y;
  A.d_planes = d_planes;
  A.d_palette_part = (f->heads & NFI_HEAD_RGB_SIGMOID) ? nullptr : d_palette_part;
  A.d_x = d_x;
  const long long jobs = nfi_sampler_chunks(B, P);
  nfi::sampler_bwd_kernel<<<(unsigned)((jobs + 3) / 4), 256, 0, (hipStream_t)stream>>>(A);
  NFI_CHECK_LAUNCH("sampler_bwd_kernel");
  return NFI_OK;
}

}  // extern "C"

// Profiling builds only (-DNFI_STAMPS): per-phase cycle sums, summed over slots, then reset.
extern "C" int32_t nfi_debug_stamps(uint64_t* out) {
#ifdef NFI_STAMPS
  static unsigned long long h[nfi::STAMP_SLOTS * nfi::STAMP_PHASES];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(nfi::nfi_stamp_acc), sizeof(h)) != hipSuccess) return NFI_ELAUNCH;
  for (int p = 0; p < nfi::STAMP_PHASES; ++p) {
    unsigned long long t = 0;
    for (int k = 0; k < nfi::STAMP_SLOTS; ++k) t += h[k * nfi::STAMP_PHASES + p];
    out[p] = t;
  }
  memset(h, 0, sizeof(h));
  if (hipMemcpyToSymbol(HIP_SYMBOL(nfi::nfi_stamp_acc), h, sizeof(h)) != hipSuccess) return NFI_ELAUNCH;
  return NFI_OK;
#else
  (void)out;
  return NFI_EINVAL;
#endif
}
