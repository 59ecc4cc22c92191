// Batched fp32 GEMM on the f16 matrix cores at fp32 accuracy (the split of DESIGN.md §3's decoder,
// applied to the Winograd products of the inversion step's caller side):
//
//   C[b] (M x N) = A[b] (M x K) . B[b] (K x N),     fp32 in, fp32 out, b < batch
//
// Every fp32 operand v, times a power of two (exact), is carried as hi = f16(v), lo = f16(v - hi);
// one fp32 product is three f16 products lo.hi + hi.lo + hi.hi on an fp32 accumulator
// (v_mfma_f32_16x16x32_f16, 16x the fp32 MFMA rate per product): the error of an fp32 dot product
// (3 2^-22 |a||b| per product at worst, below the K 2^-24 accumulation bound for K >= 12; K here is
// the channel count, 64..512).  Scales: A (frozen Winograd weights U) per batch entry, computed once
// when A is split (nfi_split16_pack: largest |A[b]| to [2^14, 2^15)); B (the input transform V) one
// scale PER IMAGE, from the running maxima its producer leaves in that image's slots (split_slot,
// nfi_common.h; nfi_wino_input_transform_max, nfi_absmax_slots): column n of B[b] belongs to image
// n / cols_per_image (the Winograd products: the image's tiles), or to image b (shared-A products: one
// image per batch entry).  Each thread splits its own column with its image's scale and the epilogue
// unscales per column, so an image's result does not depend on the other images of its batch (a
// sharded run gives each image the operand precision of the unsharded one).  An operand 2^-k below its
// image's maximum is exact to 2^-(39-k) of itself — fp32-level to k ~ 15 and, beyond, below the
// Winograd transform's own rounding (a few 1e-6 of the largest output, tests/test_gpu_conv.py).
//
// Tiling: a 256-thread workgroup computes a 128 x 128 tile of C, each wave 64 x 64 (4 x 4 blocks of
// 16 x 16, 16 accumulators of 4 floats); K in steps of 32 (one f16 MFMA deep).  Per step the
// workgroup stages A's hi / lo rows (pre-split in HBM: 16 KB) and B's 32 x 128 fp32 slab, split in
// registers on its way to LDS as B^T hi / lo rows (each thread: one column, 16 consecutive k —
// coalesced 256-B row reads across the wave), 40 KB of LDS; the next step's global loads are in
// flight during the step's 48 MFMAs per wave.  Rows padded by 8 halves (80 B) so the b128 operand
// reads of 16 lanes spread over the banks.  Measured against the alternatives kept for A/B
// (scripts/gemm_bench.py, profiles/r04_gemm_bench.log): 256 x 128 / 128 x 256 tiles of 8 waves
// (NFI_GEMM_TILE=42 / 24) 0-50 % slower, 2 x 2 waves of 128 x 128 (NFI_GEMM_TILE=88: half the LDS
// operand bytes per MFMA, 256 accumulation registers, one wave per SIMD) 20-100 % slower, two register
// stages of prefetch (NFI_GEMM_PF=2: occupancy 2) 0-15 % slower, a wide-load kernel (8 x 4 B blocks
// per thread, removed in round 6) 5-25 % slower; 200-256 TFLOP/s
// fp32-equivalent on the 256-512-channel Winograd shapes, 2x hipBLASLt's fp32 bmm.
#include <algorithm>
#include <cstdlib>

#include "nfi_common.h"
#include "nfi_host.h"
#include "../../include/nfi_producer.h"

namespace nfi {
namespace gemm {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
// NFI_GEMM_BUF 1: the general kernel's operands through buffer loads (32-bit offsets, out-of-range rows
// and columns read as zeros) and B split by v_cvt_pk_f16_f32 + v_fma_mix; 0: flat loads + selects
#ifndef NFI_GEMM_BUF
#define NFI_GEMM_BUF 1
#endif
constexpr int LDK = BK + 8;                    // halves per LDS row (80 B)

__device__ __forceinline__ f4v mfma_h(u4v a, u4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}

// s = 2^e, inv = 2^-e with m s in [2^14, 2^15) (e = 0 for m = 0 or not finite)
__device__ __forceinline__ void pow2_scale15(float m, float& s, float& inv) {
  int e = 15 - __builtin_amdgcn_frexp_expf(m);
  e = (m > 0.f && m < __builtin_inff()) ? min(max(e, -120), 120) : 0;
  s = __builtin_ldexpf(1.f, e);
  inv = __builtin_ldexpf(1.f, -e);
}

__device__ __forceinline__ unsigned short h_bits(float v) { return __builtin_bit_cast(unsigned short, (_Float16)v); }
__device__ __forceinline__ float h_val(unsigned short b) { return (float)__builtin_bit_cast(_Float16, b); }

// ---- A: split once (frozen weights) --------------------------------------------------------------
// one workgroup per batch entry: the largest |A[b]|, then hi / lo halves of A[b] * 2^e and 2^-e
__global__ void __launch_bounds__(256) split_pack_kernel(const float* __restrict__ A, long long per,
                                                         unsigned short* __restrict__ Ah,
                                                         unsigned short* __restrict__ Al, float* __restrict__ inv) {
  __shared__ float red[4];
  const long long b = blockIdx.x;
  const float* a = A + b * per;
  float m = 0.f;
  for (long long i = threadIdx.x; i < per; i += 256) m = fmaxf(m, fabsf(a[i]));
  m = wave_max(m);
  if (lane_id() == 0) lds_st_fenced(red + (threadIdx.x >> 6), m);
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s, is;
  pow2_scale15(m, s, is);
  for (long long i = threadIdx.x; i < per; i += 256) {
    const float v = a[i] * s;
    const unsigned short h = h_bits(v);
    Ah[b * per + i] = h;
    Al[b * per + i] = h_bits(v - h_val(h));
  }
  if (threadIdx.x == 0) inv[b] = is;
}

// ---- the product ---------------------------------------------------------------------------------
struct Args {
  const unsigned short* Ah;   // [batch][M][K] f16 bits
  const unsigned short* Al;
  const float* a_inv;         // [batch]
  const float* B;             // [batch][K][N]
  const unsigned* b_max;      // [SPLIT_SLOTS + 1] per-image running maxima of |B| (float bits) + counter
  float* C;                   // [batch][M][N]
  int M, N, K;
  int a_shared;               // 1: one A (and scale) for every batch entry
  int ksplit, kchunk;         // (general kernel) K in ksplit ranges of kchunk: blockIdx.z = b ksplit + s,
  float* work;                //   range s's partial C to work[s][b][M][N] when ksplit > 1
  int xcd;                    // 1: XCD-major tile order (below)
  int cpi;                    // columns per image (image of column n: n / cpi; a_shared: image b)
  int nslot;                  // slots the last workgroup returns to zero (images used x SPLIT_ISLOTS)
};

// B's scale of this lane's image (images non-decreasing across the wave's lanes): per image of the
// wave, its 64 slots read one per lane and reduced across the wave
__device__ __forceinline__ void image_scale(const unsigned* b_max, int img, float& s, float& inv) {
  static_assert(SPLIT_ISLOTS == 64, "one slot per lane");
  const int i0 = __builtin_amdgcn_readfirstlane(img);
  const int i1 = __builtin_amdgcn_readlane(img, 63);
  float mine = 0.f;
  if (i0 == i1) {   // (wave-uniform) the wave's columns in one image: one load per lane
    mine = wave_max_dpp(__uint_as_float(b_max[split_slot(i0, lane_id())]));
  } else {
    for (int i = i0; i <= i1; i += 4) {   // (four images' loads in flight per pass: small maps span many)
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __uint_as_float(b_max[split_slot(min(i + u, i1), lane_id())]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float m = wave_max_dpp(v[u]);
        if (img == i + u) mine = m;
      }
    }
  }
  pow2_scale15(mine, s, inv);
}

// The B maxima are consumed, not copied: the used slots of b_max (float bits) + b_max[SPLIT_SLOTS] (a
// completion counter) return to zero when the launch's last workgroup finishes, so the producer of the
// next maxima needs no memset launch.  Every workgroup read b_max at its start, before its first
// barrier; the one whose increment completes the count runs after all of those reads.  Relaxed
// atomics, no fence: a release fence at agent scope writes back the L2 (measured: the inversion step
// 16 -> 20 ms).
__device__ __forceinline__ void release_slots(const unsigned* b_max, int nslot) {
  __shared__ int last;
  __syncthreads();
  unsigned* bm = const_cast<unsigned*>(b_max);
  if (threadIdx.x == 0) {
    const unsigned total = gridDim.x * gridDim.y * gridDim.z;
    last = __hip_atomic_fetch_add(bm + SPLIT_SLOTS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
  }
  __syncthreads();
  if (last) {
    for (int i = threadIdx.x; i < nslot; i += blockDim.x)
      __hip_atomic_store(bm + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(bm + SPLIT_SLOTS, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Workgroups are dispatched round-robin over the 8 XCDs in linear order (x fastest), each XCD with
// its own L2.  XCD-major order: the tiles an XCD runs are a contiguous range of (n block fastest, m
// block, batch entry), so the tiles sharing an A row block or a B column slab meet in one L2 instead of
// eight (bijective for any tile count: the first T mod 8 XCDs take one tile more).
__device__ __forceinline__ void tile_order(int xcd, int& bx, int& by, int& bz) {
  bx = blockIdx.x;
  by = blockIdx.y;
  bz = blockIdx.z;
  if (!xcd) return;
  const unsigned gx = gridDim.x, gy = gridDim.y, T = gx * gy * gridDim.z;
  const unsigned L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned x = L & 7, q = T >> 3, r = T & 7;
  const unsigned t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
  bx = (int)(t % gx);
  by = (int)((t / gx) % gy);
  bz = (int)(t / (gx * gy));
}

// WM x WN waves of 64 x 64: tile (64 WM) x (64 WN), 64 WM WN threads
// RX x RY blocks of 16 x 16 per wave (4 x 4: 64 accumulator registers; 8 x 8: the 256 of the
// accumulation registers, one wave per SIMD, half the LDS operand bytes per MFMA)
template <int WM, int WN, int PF, int RX = 4, int RY = 4>
__global__ void __launch_bounds__(64 * WM * WN, RX * RY > 32 ? 1 : RX * RY > 16 ? 2 : (WM * WN == 4 ? (PF == 1 ? 3 : 2) : 1))
    split16_gemm_kernel(Args g) {
  constexpr int T = 64 * WM * WN, TBM = 16 * RX * WM, TBN = 16 * RY * WN;
  constexpr int CA = TBM * 4 / T;    // 8-half chunks of A's K-step rows per thread (hi; as many lo)
  constexpr int KB = 32 * TBN / T;   // k rows of B's slab per thread (one column)
  static_assert(CA >= 1 && CA <= 4 && KB >= 8 && KB <= 32 && KB % 8 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * LDK * (TBM + TBN)];   // A hi, A lo, Bt hi, Bt lo
  unsigned short* Ahs = lds;
  unsigned short* Als = lds + TBM * LDK;
  unsigned short* Bhs = lds + 2 * TBM * LDK;
  unsigned short* Bls = Bhs + TBN * LDK;
  const int tid = threadIdx.x, l = lane_id(), wv = tid >> 6;
  int bx, by, bz;
  tile_order(g.xcd, bx, by, bz);
  const int b = bz / g.ksplit, ks = bz - b * g.ksplit;
  const int m0 = by * TBM, n0 = bx * TBN;
  const int M = g.M, N = g.N, K = g.K;
  const int kbeg = ks * g.kchunk, kend = min(K, kbeg + g.kchunk);
  const int ba = g.a_shared ? 0 : b;

  const unsigned short* Ahg = g.Ah + (long long)ba * M * K;
  const unsigned short* Alg = g.Al + (long long)ba * M * K;
  const float* Bg = g.B + (long long)b * K * N;

  // global -> register staging: A (row ar, halves ak .. ak + 8 CA - 1 of the K-step: CA b128 loads
  // each of hi and lo), B column bn, k = bk .. bk + KB - 1 (coalesced rows across the wave)
  const int ar = (tid * CA) >> 2, ak = 8 * ((tid * CA) & 3);
  const bool a_ok = m0 + ar < M;
  const int bn = tid % TBN, bk = (tid / TBN) * KB;
  const int bcol = min(n0 + bn, N - 1);
  const bool b_ok = n0 + bn < N;
  // B's scale: this thread's column's image; the epilogue unscales each column by its own (the
  // column scales go through the operand LDS once the K loop is done: a separate array would take
  // the LDS past 4 workgroups per CU)
  float sb, isb;
  image_scale(g.b_max, g.a_shared ? b : bcol / g.cpi, sb, isb);
#if NFI_GEMM_BUF
  // Buffer loads on the batch entry's A halves and B: 32-bit offsets (no 64-bit address arithmetic
  // per load), the K-step and the row i of B in the scalar offset, and rows / columns past the matrix
  // given an offset at the buffer's end, so they load zeros (no selects)
  const __amdgpu_buffer_rsrc_t rah = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(Ahg), (short)0,
                                                                       M * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ral = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(Alg), (short)0,
                                                                       M * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bg), (short)0, K * N * 4,
                                                                       0x00020000);
  const int va = a_ok ? ((m0 + ar) * K + ak) * 2 : M * K * 2;
  const int vb = b_ok ? (bk * N + n0 + bn) * 4 : K * N * 4;
  u4v RA[PF][2 * CA];
  float RB[PF][KB];
  auto load = [&](int k0, u4v (&ra)[2 * CA], float (&rb)[KB]) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      ra[i] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rah, va + 16 * i, k0 * 2, 0));
      ra[CA + i] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(ral, va + 16 * i, k0 * 2, 0));
    }
#pragma unroll
    for (int i = 0; i < KB; ++i)
      rb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbs, vb, (k0 + i) * N * 4, 0));
  };
  auto store = [&](const u4v (&ra)[2 * CA], const float (&rb)[KB]) {
    u4v* dh = reinterpret_cast<u4v*>(Ahs + ar * LDK + ak);
    u4v* dl = reinterpret_cast<u4v*>(Als + ar * LDK + ak);
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      lds_st_fenced(dh + i, ra[i]);
      lds_st_fenced(dl + i, ra[CA + i]);
    }
    // hi = f16(v), lo = f16(v - hi) of v = B sb, two values per register: v_cvt_pk_f16_f32 for hi,
    // v_fma_mix (f16(hi * -1 + v)) for lo into a copy of hi (a register the compiler writes itself)
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    u4v hv[KB / 8], lv[KB / 8];
#pragma unroll
    for (int i = 0; i < KB; i += 2) {
      const float v0 = rb[i] * sb, v1 = rb[i + 1] * sb;
      const unsigned h = __builtin_bit_cast(unsigned, h2v{(_Float16)v0, (_Float16)v1});
      unsigned o = h;
      asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
          : "+v"(o) : "v"(h), "v"(v0), "v"(v1));
      hv[i >> 3][(i >> 1) & 3] = h;
      lv[i >> 3][(i >> 1) & 3] = o;
    }
    u4v* eh = reinterpret_cast<u4v*>(Bhs + bn * LDK + bk);
    u4v* el = reinterpret_cast<u4v*>(Bls + bn * LDK + bk);
#pragma unroll
    for (int i = 0; i < KB / 8; ++i) {
      lds_st_fenced(eh + i, hv[i]);
      lds_st_fenced(el + i, lv[i]);
    }
  };
#else
  const int arow = min(m0 + ar, M - 1);
  u4v RA[PF][2 * CA];
  float RB[PF][KB];
  auto load = [&](int k0, u4v (&ra)[2 * CA], float (&rb)[KB]) {
    const u4v* ph = reinterpret_cast<const u4v*>(Ahg + (long long)arow * K + k0 + ak);
    const u4v* pl = reinterpret_cast<const u4v*>(Alg + (long long)arow * K + k0 + ak);
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      ra[i] = ph[i];
      ra[CA + i] = pl[i];
    }
    const float* pb = Bg + (long long)(k0 + bk) * N + bcol;
#pragma unroll
    for (int i = 0; i < KB; ++i) rb[i] = pb[(long long)i * N];
  };
  auto store = [&](const u4v (&ra)[2 * CA], const float (&rb)[KB]) {
    const u4v z = {0u, 0u, 0u, 0u};
    u4v* dh = reinterpret_cast<u4v*>(Ahs + ar * LDK + ak);
    u4v* dl = reinterpret_cast<u4v*>(Als + ar * LDK + ak);
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      lds_st_fenced(dh + i, a_ok ? ra[i] : z);
      lds_st_fenced(dl + i, a_ok ? ra[CA + i] : z);
    }
    u4v hv[KB / 8], lv[KB / 8];
#pragma unroll
    for (int i = 0; i < KB; i += 2) {
      const float v0 = b_ok ? rb[i] * sb : 0.f, v1 = b_ok ? rb[i + 1] * sb : 0.f;
      const unsigned short h0 = h_bits(v0), h1 = h_bits(v1);
      const unsigned short l0 = h_bits(v0 - h_val(h0)), l1 = h_bits(v1 - h_val(h1));
      hv[i >> 3][(i >> 1) & 3] = (unsigned)h0 | ((unsigned)h1 << 16);
      lv[i >> 3][(i >> 1) & 3] = (unsigned)l0 | ((unsigned)l1 << 16);
    }
    u4v* eh = reinterpret_cast<u4v*>(Bhs + bn * LDK + bk);
    u4v* el = reinterpret_cast<u4v*>(Bls + bn * LDK + bk);
#pragma unroll
    for (int i = 0; i < KB / 8; ++i) {
      lds_st_fenced(eh + i, hv[i]);
      lds_st_fenced(el + i, lv[i]);
    }
  };
#endif

  // wave (wm, wn) computes rows 16 RX wm.., columns 16 RY wn.. of the tile
  const int wm = wv / WN, wn = wv % WN;
  const int i16 = l & 15, kg = l >> 4;
  f4v acc[RX][RY];
#pragma unroll
  for (int x = 0; x < RX; ++x)
#pragma unroll
    for (int y = 0; y < RY; ++y) acc[x][y] = f4v{0.f, 0.f, 0.f, 0.f};

  auto compute = [&]() {
    u4v ah[RX], al[RX];
#pragma unroll
    for (int x = 0; x < RX; ++x) {
      const int r = (16 * RX * wm + 16 * x + i16) * LDK + 8 * kg;
      ah[x] = *reinterpret_cast<const u4v*>(Ahs + r);
      al[x] = *reinterpret_cast<const u4v*>(Als + r);
    }
#pragma unroll
    for (int y = 0; y < RY; ++y) {
      const int r = (16 * RY * wn + 16 * y + i16) * LDK + 8 * kg;
      const u4v bh = *reinterpret_cast<const u4v*>(Bhs + r);
      const u4v bl = *reinterpret_cast<const u4v*>(Bls + r);
#pragma unroll
      for (int x = 0; x < RX; ++x) {
        acc[x][y] = mfma_h(al[x], bh, acc[x][y]);   // small terms first
        acc[x][y] = mfma_h(ah[x], bl, acc[x][y]);
        acc[x][y] = mfma_h(ah[x], bh, acc[x][y]);
      }
    }
  };
  // PF register stages: the loads of step k + PF are issued once step k's registers are in LDS and
  // are in flight during PF steps' products
  auto step = [&](int k0, u4v (&ra)[2 * CA], float (&rb)[KB]) {
    store(ra, rb);
    __syncthreads();
    if (k0 + PF * BK < kend) load(k0 + PF * BK, ra, rb);
    compute();
    __syncthreads();
  };
  load(kbeg, RA[0], RB[0]);
  if constexpr (PF == 1) {
    for (int k0 = kbeg; k0 < kend; k0 += BK) step(k0, RA[0], RB[0]);
  } else {
    if (kbeg + BK < kend) load(kbeg + BK, RA[PF - 1], RB[PF - 1]);
    int k0 = kbeg;
    for (; k0 + BK < kend; k0 += 2 * BK) {
      step(k0, RA[0], RB[0]);
      step(k0 + BK, RA[PF - 1], RB[PF - 1]);
    }
    if (k0 < kend) step(k0, RA[0], RB[0]);
  }
  // C rows m0 + 16 RX wm + 16 x + 4 kg + r, column n0 + 16 RY wn + 16 y + i16
  float* col_scale = reinterpret_cast<float*>(lds);   // (the K loop ended on a barrier)
  if (tid < TBN) col_scale[bn] = g.a_inv[ba] * isb;
  __syncthreads();
  float* Cg = (g.ksplit > 1 ? g.work + (long long)ks * (gridDim.z / g.ksplit) * M * N : g.C) + (long long)b * M * N;
#if NFI_GEMM_BUF
  if (m0 + TBM <= M && n0 + TBN <= N) {   // (workgroup-uniform) an interior tile: no bounds tests, buffer
                                          // stores at 32-bit offsets (rows 16 apart in the scalar offset)
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(Cg, (short)0, M * N * 4, 0x00020000);
    const int vc = ((m0 + 16 * RX * wm + 4 * kg) * N + n0 + 16 * RY * wn + i16) * 4;
    float cs[RY];
#pragma unroll
    for (int y = 0; y < RY; ++y) cs[y] = col_scale[16 * RY * wn + 16 * y + i16];
#pragma unroll
    for (int x = 0; x < RX; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int y = 0; y < RY; ++y)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[x][y][r] * cs[y]), rc, vc + 64 * y,
                                                (16 * x + r) * N * 4, 0);
  } else
#endif
  {
#pragma unroll
    for (int x = 0; x < RX; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 16 * RX * wm + 16 * x + 4 * kg + r;
        if (m >= M) continue;
#pragma unroll
        for (int y = 0; y < RY; ++y) {
          const int n = n0 + 16 * RY * wn + 16 * y + i16;
          if (n < N) Cg[(long long)m * N + n] = acc[x][y][r] * col_scale[n - n0];
        }
      }
  }
  release_slots(g.b_max, g.nslot);
}

// C = sum over s of work[s] (fixed order: deterministic), float4 per thread
__global__ void __launch_bounds__(256) ksum_kernel(const float* __restrict__ work, float* __restrict__ C, long long n4,
                                                    int ksplit) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  f4v a = reinterpret_cast<const f4v*>(work)[i];
  for (int s = 1; s < ksplit; ++s) a += reinterpret_cast<const f4v*>(work)[(long long)s * n4 + i];
  reinterpret_cast<f4v*>(C)[i] = a;
}

// running maximum of |x| per image, x [nimg][per], into the images' slots (generic callers; the
// Winograd input transform keeps its own, nfi_conv.hip).  grid (blocks per image, nimg)
// STORE: a grid of exactly SPLIT_ISLOTS blocks per image (<= SPLIT_IMAGES images), block j writing
// slot j of its image (every slot of the used images written: no memset) and block (0, 0) the
// completion counter's zero; else atomicMax into zeroed slots
template <bool STORE>
__global__ void __launch_bounds__(256) absmax_kernel(const float* __restrict__ x, long long per,
                                                     unsigned* __restrict__ slots) {
  __shared__ float red[4];
  const float* xi = x + (long long)blockIdx.y * per;
  float m = 0.f;
  const long long stride = (long long)gridDim.x * 256;
  if ((per & 3) == 0 && ((uintptr_t)x & 15) == 0) {   // float4 loads, four in flight per thread
    const float4* x4 = reinterpret_cast<const float4*>(xi);
    const long long n4 = per >> 2;
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u) m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = x4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < per; i += stride) m = fmaxf(m, fabsf(xi[i]));
  }
  m = wave_max(m);
  if (lane_id() == 0) lds_st_fenced(red + (threadIdx.x >> 6), m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned v = __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
    if constexpr (STORE) {
      slots[split_slot(blockIdx.y, blockIdx.x)] = v;
      if (blockIdx.x == 0 && blockIdx.y == 0) slots[SPLIT_SLOTS] = 0u;
    } else {
      atomicMax(slots + split_slot(blockIdx.y, blockIdx.x), v);
    }
  }
}

}  // namespace gemm
}  // namespace nfi

using namespace nfi;

extern "C" {

int32_t nfi_split16_pack(const float* A, int32_t batch, int64_t per, uint16_t* Ah, uint16_t* Al, float* a_inv,
                         void* stream) {
  NFI_REQUIRE(A && Ah && Al && a_inv, "split16_pack: null pointer");
  NFI_REQUIRE(batch > 0 && per > 0, "split16_pack: bad shape batch=%d per=%lld", batch, (long long)per);
  hipLaunchKernelGGL(gemm::split_pack_kernel, dim3(batch), dim3(256), 0, (hipStream_t)stream, A, (long long)per, Ah,
                     Al, a_inv);
  NFI_CHECK_LAUNCH("split_pack_kernel");
  return NFI_OK;
}

static_assert(NFI_SPLIT16_SLOT_WORDS == SPLIT_SLOTS + 1, "include/nfi_producer.h slot words");
int32_t nfi_split16_slot_words(void) { return SPLIT_SLOTS + 1; }

int32_t nfi_absmax_slots(const float* x, int32_t nimg, int64_t per_image, uint32_t* slots, void* stream) {
  NFI_REQUIRE(x && slots && nimg > 0 && nimg <= 65535 && per_image > 0, "absmax_slots: bad arguments");
  if (nimg >= 4096 / SPLIT_ISLOTS && nimg <= SPLIT_IMAGES) {   // (64-256 images) one block per slot: no memset
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::absmax_kernel<true>), dim3(SPLIT_ISLOTS, (unsigned)nimg), dim3(256), 0,
                       (hipStream_t)stream, x, (long long)per_image, slots);
  } else {
    NFI_REQUIRE(hipMemsetAsync(slots, 0, (SPLIT_SLOTS + 1) * 4, (hipStream_t)stream) == hipSuccess, "absmax_slots: memset");
    const long long blocks = std::max<long long>(1, std::min<long long>((per_image + 255) / 256, 4096 / nimg));
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::absmax_kernel<false>), dim3((unsigned)blocks, (unsigned)nimg), dim3(256), 0,
                       (hipStream_t)stream, x, (long long)per_image, slots);
  }
  NFI_CHECK_LAUNCH("absmax_kernel");
  return NFI_OK;
}

static int32_t gemm_split16_impl(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                                 const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                                 int32_t cpi, int a_shared, int32_t ksplit, float* work, void* stream) {
  NFI_REQUIRE(Ah && Al && a_inv && B && b_max && C, "gemm_split16: null pointer");
  NFI_REQUIRE(a_shared || (cpi > 0 && N % cpi == 0), "gemm_split16: cols_per_image=%d must divide N=%d", cpi, N);
  NFI_REQUIRE(batch > 0 && batch <= 65535 && M > 0 && N > 0 && K > 0 && K % gemm::BK == 0,
              "gemm_split16: bad shape batch=%d M=%d N=%d K=%d (K a multiple of %d)", batch, M, N, K, gemm::BK);
  // (each operand and result matrix addressed by 32-bit byte offsets: buffer loads / stores)
  NFI_REQUIRE((long long)M * K * 2 < (1ll << 31) && (long long)K * N * 4 < (1ll << 31) && (long long)M * N * 4 < (1ll << 31),
              "gemm_split16: matrix too large (each operand < 2 GiB)");
  NFI_REQUIRE(((uintptr_t)Ah & 15) == 0 && ((uintptr_t)Al & 15) == 0, "gemm_split16: A halves must be 16-B aligned");
  gemm::Args g{reinterpret_cast<const unsigned short*>(Ah), reinterpret_cast<const unsigned short*>(Al), a_inv, B,
               b_max, C, M, N, K, a_shared, 1, K, nullptr, 1, a_shared ? N : cpi, 0};
  const int nimg = a_shared ? batch : N / cpi;
  g.nslot = std::min(nimg, SPLIT_IMAGES) * SPLIT_ISLOTS;
  // XCD-major tile order where a row of tiles is short (<= 8 column blocks: the 512-channel layers'
  // products, 5-12 % faster); the long rows of the large maps stream better in linear order (3-6 %,
  // profiles/r04_gemm_bench.log).  NFI_GEMM_XCD=0/1 forces it (A/B).
  const char* xe = getenv("NFI_GEMM_XCD");
  g.xcd = xe ? atoi(xe) : 0;
  NFI_REQUIRE(ksplit >= 1 && (ksplit == 1 || work), "gemm_split16: ksplit=%d needs a workspace", ksplit);
  // tile of the general kernel: WM x WN waves (NFI_GEMM_TILE = "WMWN": 22 default, 42, 24, 41, 14)
  const char* te = getenv("NFI_GEMM_TILE");
  // (48: 64 x 128 waves, a 128 x 256 tile at occupancy 2 with a quarter fewer LDS bytes per MFMA:
  //  3-9 % faster than 22 alone on the long products (N >= 16384), 10-20 % slower on the rest, and
  //  the vgg inversion step with it on those products 15.76-15.82 vs 15.58-15.64 ms: not the default)
  const int tile = te ? atoi(te) : 22;
  const int WM = tile / 10, WN = tile % 10;
  NFI_REQUIRE(tile == 22 || tile == 42 || tile == 24 || tile == 41 || tile == 14 || tile == 88 || tile == 48,
              "gemm_split16: NFI_GEMM_TILE=%d", tile);
  // (88: 2 x 2 waves of 128 x 128 — a 256 x 256 tile; 48: 2 x 2 waves of 64 x 128)
  const int TM = tile == 88 ? 256 : tile == 48 ? 128 : 64 * WM;
  const int TN = tile == 88 || tile == 48 ? 256 : 64 * WN;
  const dim3 grid((unsigned)((N + TN - 1) / TN), (unsigned)((M + TM - 1) / TM), (unsigned)batch);
  NFI_REQUIRE(grid.y <= 65535, "gemm_split16: M too large");
  if (!xe) g.xcd = grid.x <= 8;
  const char* pe = getenv("NFI_GEMM_PF");   // register prefetch depth (A/B: 1 or 2)
  const int pf = pe ? atoi(pe) : 1;
  auto general = [&](dim3 gr) {
    if (pf == 2) {
      hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<2, 2, 2>), gr, dim3(256), 0, (hipStream_t)stream, g);
      return;
    }
    switch (tile) {
      case 88: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<2, 2, 1, 8, 8>), gr, dim3(256), 0, (hipStream_t)stream, g); break;
      case 48: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<2, 2, 1, 4, 8>), gr, dim3(256), 0, (hipStream_t)stream, g); break;
      case 42: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<4, 2, 1>), gr, dim3(512), 0, (hipStream_t)stream, g); break;
      case 24: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<2, 4, 1>), gr, dim3(512), 0, (hipStream_t)stream, g); break;
      case 41: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<4, 1, 1>), gr, dim3(256), 0, (hipStream_t)stream, g); break;
      case 14: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<1, 4, 1>), gr, dim3(256), 0, (hipStream_t)stream, g); break;
      default: hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm::split16_gemm_kernel<2, 2, 1>), gr, dim3(256), 0, (hipStream_t)stream, g); break;
    }
  };
  if (ksplit > 1) {   // K ranges of whole steps, partials summed in order
    const int steps = K / gemm::BK;
    // ranges of ceil(steps / ksplit) steps, and only as many ranges as that covers: no range is
    // empty (K = 160, ksplit 4: 5 steps -> 3 ranges of 2, 2, 1 steps; the kernel's first load of a
    // range reads at its start unconditionally)
    const int per = (steps + std::min(ksplit, steps) - 1) / std::min(ksplit, steps);
    ksplit = (steps + per - 1) / per;
    g.ksplit = ksplit;
    g.kchunk = per * gemm::BK;
    g.work = work;
    NFI_REQUIRE((long long)batch * ksplit <= 65535, "gemm_split16: batch x ksplit too large");
    NFI_REQUIRE(((uintptr_t)work & 15) == 0 && ((uintptr_t)C & 15) == 0 && (long long)M * N % 4 == 0,
                "gemm_split16: ksplit needs 16-B aligned work / C and M N % 4 == 0");
    general(dim3(grid.x, grid.y, (unsigned)(batch * ksplit)));
    NFI_CHECK_LAUNCH("split16_gemm_kernel");
    const long long n4 = (long long)batch * M * N / 4;
    hipLaunchKernelGGL(gemm::ksum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, work, C,
                       n4, ksplit);
    NFI_CHECK_LAUNCH("ksum_kernel");
  } else {
    general(grid);
    NFI_CHECK_LAUNCH("split16_gemm_kernel");
  }
  return NFI_OK;
}

// The maxima slots are consumed by the launch's last workgroup.  A call that returns an error has
// not consumed them (rejected before the launch) or may not have (a failed launch): they are zeroed
// here on the same stream, so the next producer's maxima start from zero instead of max(stale, new) —
// a stale larger maximum would silently coarsen the next product's B scale
// (tests/test_gpu_gemm.py::test_maxima_slots_back_to_back_and_after_rejection).
static int32_t gemm_split16(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                            const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                            int32_t cpi, int a_shared, int32_t ksplit, float* work, void* stream) {
  const int32_t rc = gemm_split16_impl(Ah, Al, a_inv, B, b_max, C, batch, M, N, K, cpi, a_shared, ksplit, work, stream);
  if (rc != NFI_OK && b_max)
    (void)hipMemsetAsync(const_cast<uint32_t*>(b_max), 0, (SPLIT_SLOTS + 1) * sizeof(uint32_t), (hipStream_t)stream);
  return rc;
}

int32_t nfi_gemm_split16(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                         const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                         int32_t cols_per_image, void* stream) {
  return gemm_split16(Ah, Al, a_inv, B, b_max, C, batch, M, N, K, cols_per_image, 0, 1, nullptr, stream);
}

int32_t nfi_gemm_split16_ksplit(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                                const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                                int32_t cols_per_image, int32_t ksplit, float* work, void* stream) {
  return gemm_split16(Ah, Al, a_inv, B, b_max, C, batch, M, N, K, cols_per_image, 0, ksplit, work, stream);
}

int32_t nfi_gemm_split16_shared_a(const uint16_t* Ah, const uint16_t* Al, const float* a_inv, const float* B,
                                  const uint32_t* b_max, float* C, int32_t batch, int32_t M, int32_t N, int32_t K,
                                  int32_t ksplit, float* work, void* stream) {
  return gemm_split16(Ah, Al, a_inv, B, b_max, C, batch, M, N, K, 0, 1, ksplit, work, stream);
}

}  // extern "C"
