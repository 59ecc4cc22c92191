// Direct 3x3 convolution (stride 1, padding 1, NCHW fp32) on the f16 matrix cores at fp32 accuracy,
// for the large-map layers of the inversion step's LPIPS VGG16 trunk (lpips 0.1 via
// lib/metrics.py:107; F.conv2d(x, w, b, padding=1) in fp32 with TF32 off, run.py:59-60) — their
// forward with the VGG block's bias + ReLU (+ 2x2 max pool) epilogue and their data gradient (the
// correlation with the rot180 / channel-swapped weight), optionally through the ReLU mask of the
// block's output (threshold_backward folded into the staging).
//
//   y[n][o][r][c] = sum_{i, ky, kx} w[o][i][ky][kx] x[n][i][r + ky - 1][c + kx - 1]
//
// As a GEMM per image: M = output channels, N = pixels, K = 9 taps x input channels.  Every fp32
// operand, times a power of two, is hi = f16(v) + lo = f16(v - hi); one product is lo.hi + hi.lo +
// hi.hi on v_mfma_f32_32x32x16_f16 (the split of nfi_gemm.hip: 3 2^-22 |a||b| per product at
// worst).  Scales: the weight one power of two (packed once per frozen weight, nfi_dconv_pack), x
// one PER IMAGE from its maxima slots (split_slot, nfi_host.h; nfi_absmax_slots), so an image's
// result does not depend on the other images of the batch.
//
// Why not Winograd here (nfi_conv.hip): on a 64 -> 64 map of 128^2 (64 images) the three-pass form
// streams V and M (2.25x the activations each way) through HBM and the fused kernel holds 288
// accumulators per lane at one wave per SIMD on the fp32 MFMA (46-64 TFLOP/s); the direct form
// moves only x and y and runs 9 x the f16 products of one fp32 product on the 2.5-PFLOP/s pipe.
//
// Workgroup: 512 threads (8 waves, two per SIMD), persistent, one per CU (159,744 B of LDS).  A tile
// is 64 output channels x 8 rows x 64 columns of one image; wave w computes channels 32 (w & 1) ..
// +31 of rows 2 (w >> 1), +1 (2 x 2 blocks of 32 x 32: 64 accumulators).  K in chunks of 16 input
// channels, two LDS chunk buffers: while the 9 taps x 12 MFMAs of every wave read one, the next
// chunk (the next tile's first after the last) goes into the other — its weights (pre-split,
// [tap][k-group][channel]) by global_load_lds, its 10 x 66-pixel region of x through registers, split
// to [k-group][pixel][8 channels] f16 planes (a b128 operand read of 16 lanes touches 16 consecutive
// 16-B slots: conflict-free at any tap shift) in three rounds placed behind the MFMAs of taps 6-8, so
// the split's vector instructions issue in the MFMAs' shadow.  One barrier per chunk.  (The staging
// after the products, by every wave at once, measured MFMA busy 0.43; two 4-wave workgroups per CU
// with one buffer each, the same.)  Tiles are dealt XCD-major (an XCD's workgroups take a contiguous
// range, so neighbouring tiles' halos and a channel block's weights share its L2).
#include <algorithm>

#include "nfi_common.h"
#include "nfi_host.h"
#include "../../include/nfi_producer.h"

namespace nfi {
namespace dconv {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int TR = 8, TC = 64, CT = 64, KC = 16;   // tile rows, columns, output channels; K chunk
constexpr int RR = TR + 2, RC = TC + 2;              // staged region (halo of 1)
constexpr int NPX = RR * RC;                         // 660 pixels
constexpr int NPXP = (NPX + 15) / 16 * 16;           // 672: a k-group plane is a multiple of 256 B
constexpr int NT = 512, NW = NT / 64;
constexpr int BU = 2 * NPX;                          // (k-group, pixel) units of x per chunk
constexpr int BRD = (BU + NT - 1) / NT;              // 3 rounds
constexpr int AU = 2 * 9 * 2 * CT;                   // 16-B weight units per chunk (hi / lo, tap, k-group, channel)
constexpr int AROWS = AU / 64;                       // 36 rows of 64 units (1 KB: one LDS-DMA wave-instruction each)
// one chunk buffer, in 16-B units: x hi [2][NPXP], x lo [2][NPXP], w hi [9][2][CT], w lo [9][2][CT]
constexpr int OB_LO = 2 * NPXP, OA = 4 * NPXP, OA_LO = 9 * 2 * CT, BUFU = OA + AU;
static_assert(2 * BUFU * 16 <= 163840, "two chunk buffers in one CU's LDS");
static_assert(BRD == 3, "three staging rounds (behind taps 6, 7, 8)");
static_assert(CT == 64 && AU % 64 == 0, "weight rows of 64 channels");

// timing experiments only (wrong results; never the product build): bit 0 skips the staging of chunks
// after the first, bit 1 the epilogue's stores (one value per tile instead)
#ifndef NFI_DCONV_EXP
#define NFI_DCONV_EXP 0
#endif

#ifndef NFI_DCONV_STAUX
#define NFI_DCONV_STAUX 2   // the epilogue's stores streamed (slc): 128^2 conv1_2 0.335 -> 0.302 ms (0: A/B builds)
#endif

struct Args {
  const float* x;          // [N][Ci][H][W]
  const float* relu_y;     // null, or [N][Ci][H][W]: x taken where relu_y > 0 (threshold_backward)
  const float* xscale;     // null, or [N][Ci]: x taken times xscale[n][c] (the synthesis layers' modulation)
  const unsigned* slots;   // per-image max |x| (split_slot layout, float bits)
  const u4v* wp;           // [2 (hi, lo)][9][Ci / 8][Co] 16-B units: 8 halves = channels 8k .. 8k + 7
  const float* w_inv;      // [1]: 2^-e of the weight's split
  const float* bias;       // null (plain convolution) or [Co]: relu(conv + bias)
  float* y;                // [N][Co][H][W]
  float* pooled;           // null or [N][Co][H/2][W/2]: MaxPool2d(2, 2) of y (needs bias)
  unsigned* ymax;          // null, or per-image max |y| slots (split_slot layout; atomicMax): the next
                           // layer's x scale without a maxima pass
  int N, Ci, Co, H, W;
  int tw, th, tco, T;      // tiles per row / per column / channel blocks; total
};

// s = 2^e, inv = 2^-e with m s in [2^14, 2^15) (e = 0 for m = 0 or not finite): nfi_gemm.hip's rule
__device__ __forceinline__ void pow2_scale15(float m, float& s, float& inv) {
  int e = 15 - __builtin_amdgcn_frexp_expf(m);
  e = (m > 0.f && m < __builtin_inff()) ? min(max(e, -120), 120) : 0;
  s = __builtin_ldexpf(1.f, e);
  inv = __builtin_ldexpf(1.f, -e);
}

__device__ __forceinline__ f16v mfma32(u4v a, u4v b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}

struct Tile {
  int n, y0, x0, co0;
};
// tile t: output-channel block fastest, then column, row, image (the channel blocks of one region
// run back to back on one XCD)
__device__ __forceinline__ Tile decode(const Args& g, int t) {
  Tile d;
  const int ct = t % g.tco;
  int r = t / g.tco;
  const int tx = r % g.tw;
  r /= g.tw;
  const int ty = r % g.th;
  d.n = r / g.th;
  d.y0 = ty * TR;
  d.x0 = tx * TC;
  d.co0 = ct * CT;
  return d;
}

// the next chunk's x in registers: unit u = tid + r NT of round r is (k-group, pixel) = channels
// 8 kg .. 8 kg + 7 of one region pixel
template <bool MASK, bool SCALE = false>
struct Stage {
  float b[BRD][8];
  float m[MASK ? BRD : 1][8];
  float xs[SCALE ? KC : 1];   // the chunk's 16 channel scales (wave-uniform: scalar registers)
  float smax;
};

template <bool MASK, bool SCALE>
__device__ __forceinline__ void stage_load(const Args& g, Stage<MASK, SCALE>& st, int t, int c) {
  const Tile d = decode(g, t);
  const int tid = threadIdx.x;
  const int HW = g.H * g.W;
  const long long img = (long long)d.n * g.Ci * HW;
  const int xbytes = g.Ci * HW * 4;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x + img), (short)0, xbytes, 0x00020000);
#pragma unroll
  for (int r = 0; r < BRD; ++r) {
    const int u = tid + r * NT;
    const int kg = u >= NPX ? 1 : 0, p = u - kg * NPX;
    const int row = p / RC, col = p - row * RC;
    const int gy = d.y0 - 1 + row, gx = d.x0 - 1 + col;
    const bool ok = u < BU && gy >= 0 && gy < g.H && gx >= 0 && gx < g.W;
    // (rows / columns past the map and the surplus units: an offset past the buffer loads zeros)
    const int vo = ok ? ((8 * kg) * HW + gy * g.W + gx) * 4 : xbytes;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      st.b[r][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo, (c * KC + i) * HW * 4, 0));
    if constexpr (MASK) {
      const __amdgpu_buffer_rsrc_t ry =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.relu_y + img), (short)0, xbytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        st.m[r][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, vo, (c * KC + i) * HW * 4, 0));
    }
  }
  if constexpr (SCALE) {
    const float* xs = g.xscale + (long long)d.n * g.Ci + c * KC;
#pragma unroll
    for (int i = 0; i < KC; ++i) st.xs[i] = xs[i];
  }
  st.smax = __uint_as_float(g.slots[split_slot(d.n, lane_id())]);
}

// round R of the staged x, split with scale s into buffer dst
template <int R, bool MASK, bool SCALE>
__device__ __forceinline__ void stage_store(const Stage<MASK, SCALE>& st, float s, u4v* __restrict__ dst) {
  const int u = threadIdx.x + R * NT;
  if (u < BU) {
    const int kg = u >= NPX ? 1 : 0, p = u - kg * NPX;
    u4v hv, lv;
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      float v0 = st.b[R][i] * s, v1 = st.b[R][i + 1] * s;
      if constexpr (SCALE) {   // (x s_c) 2^e: the image scale bounds max |x s_c|
        v0 *= kg ? st.xs[8 + i] : st.xs[i];
        v1 *= kg ? st.xs[9 + i] : st.xs[i + 1];
      }
      if constexpr (MASK) {
        v0 = st.m[R][i] > 0.f ? v0 : 0.f;
        v1 = st.m[R][i + 1] > 0.f ? v1 : 0.f;
      }
      // hi = f16(v) two at a time (v_cvt_pk_f16_f32), lo = f16(v - hi) by v_fma_mix into a copy of hi
      const unsigned h = __builtin_bit_cast(unsigned, h2v{(_Float16)v0, (_Float16)v1});
      unsigned o = h;
      asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
          : "+v"(o) : "v"(h), "v"(v0), "v"(v1));
      hv[i >> 1] = h;
      lv[i >> 1] = o;
    }
    lds_st_fenced(dst + kg * NPXP + p, hv);
    lds_st_fenced(dst + OB_LO + kg * NPXP + p, lv);
  }
}

// the chunk's weights straight into the LDS (global_load_lds, 16 B per lane: no registers): row q =
// (hi / lo, tap, k-group) of 64 channels is 1 KB contiguous in the packed weight and in the LDS image,
// one wave-instruction each; wave w copies rows w, w + 8, ... (36 rows).  The chunk's barrier is
// preceded by vmcnt(0).
__device__ __forceinline__ void weights_to_lds(const Args& g, int t, int c, u4v* __restrict__ buf) {
  const int w = threadIdx.x >> 6, l = lane_id();
  const int co0 = (t % g.tco) * CT, ci8 = g.Ci / 8;
#pragma unroll
  for (int k = 0; k < (AROWS + NW - 1) / NW; ++k) {
    const int q = w + NW * k;
    if (q < AROWS) {   // (wave-uniform)
      const int hl = q / 18, tap = (q >> 1) % 9, kq = q & 1;
      const u4v* src = g.wp + ((long long)(hl * 9 + tap) * ci8 + c * (KC / 8) + kq) * g.Co + co0 + l;
      __builtin_amdgcn_global_load_lds(src, buf + OA + q * 64, 16, 0, 0);
    }
  }
}

struct Ops {
  u4v ah, al, bh[2][2], bl[2][2];
};
template <int TAP>
__device__ __forceinline__ void load_ops(const u4v* __restrict__ bx, const u4v* __restrict__ aw, Ops& o) {
  constexpr int ky = TAP / 3, kx = TAP % 3;
  o.ah = aw[TAP * 2 * CT];
  o.al = aw[OA_LO + TAP * 2 * CT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = (i + ky) * RC + 32 * j + kx;
      o.bh[i][j] = bx[q];
      o.bl[i][j] = bx[OB_LO + q];
    }
}
// per accumulator lo.hi, hi.lo, then hi.hi (small terms first); the four blocks' MFMAs interleaved so
// no MFMA waits on the one before it
__device__ __forceinline__ void tap_products(const Ops& o, f16v (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(o.al, o.bh[i][j], acc[i][j]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(o.ah, o.bl[i][j], acc[i][j]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(o.ah, o.bh[i][j], acc[i][j]);
}

// One chunk: the 9 taps of wave (cb, rp) on buffer cur — one tap's operands in flight while the
// previous tap's 12 MFMAs run (two operand sets; scheduling barriers keep further reads from being
// hoisted) — with, when `more`, the next chunk's x split into buffer nxt in three rounds behind the
// MFMAs of taps 6, 7 and 8 (its loads were issued at the chunk's start).
template <bool MASK, bool SCALE>
__device__ __forceinline__ void chunk(const u4v* __restrict__ cur, u4v* __restrict__ nxt, int cb, int rp,
                                      f16v (&acc)[2][2], const Stage<MASK, SCALE>& st, bool more, float& inv) {
  const int l = lane_id(), kg = l >> 5, lr = l & 31;
  const u4v* bx = cur + kg * NPXP + (2 * rp) * RC + lr;
  const u4v* aw = cur + OA + kg * CT + 32 * cb + lr;
  Ops o0, o1;
  load_ops<0>(bx, aw, o0);
  load_ops<1>(bx, aw, o1);
  tap_products(o0, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_ops<2>(bx, aw, o0);
  tap_products(o1, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_ops<3>(bx, aw, o1);
  tap_products(o0, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_ops<4>(bx, aw, o0);
  tap_products(o1, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_ops<5>(bx, aw, o1);
  tap_products(o0, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_ops<6>(bx, aw, o0);
  tap_products(o1, acc);   // tap 5
  __builtin_amdgcn_sched_barrier(0);
  load_ops<7>(bx, aw, o1);
  tap_products(o0, acc);   // tap 6
  __builtin_amdgcn_sched_barrier(0);
  float s = 1.f;
  if (more) {
    pow2_scale15(wave_max_dpp(st.smax), s, inv);
    stage_store<0>(st, s, nxt);
  }
  __builtin_amdgcn_sched_barrier(0);
  load_ops<8>(bx, aw, o0);
  tap_products(o1, acc);   // tap 7
  __builtin_amdgcn_sched_barrier(0);
  if (more) stage_store<1>(st, s, nxt);
  __builtin_amdgcn_sched_barrier(0);
  tap_products(o0, acc);   // tap 8
  __builtin_amdgcn_sched_barrier(0);
  if (more) stage_store<2>(st, s, nxt);
}

// accumulators -> y (x scale; EPI 1: + bias, ReLU; EPI 2: also the 2 x 2 max pool).  Lane l of block
// (i, j) holds channels co0 + 32 cb + (r & 3) + 8 (r >> 2) + 4 (l >> 5) (register r) of pixel (row
// 2 rp + i, column 32 j + (l & 31)).  Buffer stores on the tile's image: a lane offset, the register's
// channel offset in the scalar offset; the 16 bias values loaded before the first store and the pool's
// column pairs by DPP (no wait inside the store sequence).
template <int EPI>
__device__ __forceinline__ void epilogue(const Args& g, const Tile& d, int cb, int rp, const f16v (&acc)[2][2],
                                         float f, int t) {
  const int l = lane_id(), kg = l >> 5, lr = l & 31;
  const int HW = g.H * g.W, H2 = g.H >> 1, W2 = g.W >> 1, HW2 = H2 * W2;
  const long long img = (long long)d.n * g.Co;
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(g.y + img * HW, (short)0, g.Co * HW * 4, 0x00020000);
  const int c0 = d.co0 + 32 * cb + 4 * kg;   // this lane's first channel
  const int vy = (c0 * HW + (d.y0 + 2 * rp) * g.W + d.x0 + lr) * 4;
  float bias[16];
  if constexpr (EPI >= 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) bias[r] = g.bias[c0 + (r & 3) + 8 * (r >> 2)];
  }
  __amdgpu_buffer_rsrc_t rpool;
  int vp = 0;
  if constexpr (EPI == 2) {
    rpool = __builtin_amdgcn_make_buffer_rsrc(g.pooled + img * HW2, (short)0, g.Co * HW2 * 4, 0x00020000);
    vp = (c0 * HW2 + ((d.y0 >> 1) + rp) * W2 + ((d.x0 + lr) >> 1)) * 4;
  }
  float ym = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int cr = (r & 3) + 8 * (r >> 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        v[i] = acc[i][j][r] * f;
        if constexpr (EPI >= 1) v[i] = fmaxf(v[i] + bias[r], 0.f);
        ym = fmaxf(ym, fabsf(v[i]));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[i]), ry, vy + (i * g.W + 32 * j) * 4,
                                              cr * HW * 4, NFI_DCONV_STAUX);
      }
      if constexpr (EPI == 2) {
        float m = fmaxf(v[0], v[1]);
        m = fmaxf(m, dpp_mov<0xB1>(m));   // the column pair (lanes l, l ^ 1)
        if (!(lr & 1))
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m), rpool, vp + 16 * j * 4, cr * HW2 * 4, NFI_DCONV_STAUX);
      }
    }
  }
  if (g.ymax) {   // one atomic per wave and tile, spread over the image's 64 slots
    ym = wave_max_dpp(ym);
    if (l == 0) atomicMax(g.ymax + split_slot(d.n, t * NW + (threadIdx.x >> 6)), __float_as_uint(ym));
  }
}

template <bool MASK, int EPI, bool SCALE = false>
__global__ void __launch_bounds__(NT, 1) dconv_kernel(Args g) {
  __shared__ __attribute__((aligned(16))) u4v lds[2 * BUFU];
  const int w = threadIdx.x >> 6;
  const int cb = w & 1, rp = w >> 1;
  // this workgroup's tiles: XCD x = blockIdx % 8 takes the contiguous range [lo, hi) of the T tiles,
  // its k-th workgroup tiles lo + k, lo + k + G/8, ...  (G a multiple of 8; else a plain stride)
  const int G = gridDim.x, b = blockIdx.x;
  int t, tstep, tend;
  if ((G & 7) == 0) {
    const int x = b & 7, k = b >> 3, q = g.T >> 3, rr = g.T & 7;
    const int lo = x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q;
    t = lo + k;
    tstep = G >> 3;
    tend = lo + q + (x < rr ? 1 : 0);
  } else {
    t = b;
    tstep = G;
    tend = g.T;
  }
  if (t >= tend) return;   // (workgroup-uniform, before any barrier)
  const int nk = g.Ci / KC;
  Stage<MASK, SCALE> st;
  float isx_next;
  {   // the first chunk, staged before the loop
    stage_load(g, st, t, 0);
    weights_to_lds(g, t, 0, lds);
    float s;
    pow2_scale15(wave_max_dpp(st.smax), s, isx_next);
    stage_store<0>(st, s, lds);
    stage_store<1>(st, s, lds);
    stage_store<2>(st, s, lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float w_inv = g.w_inv[0];
  int cur = 0;
  for (;;) {
    const float isx = isx_next;
    f16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f16v{};
    for (int c = 0; c < nk; ++c) {
      int nt = t, nc = c + 1;
      if (nc == nk) {
        nt = t + tstep;
        nc = 0;
      }
      const bool more = (NFI_DCONV_EXP & 1) ? false : nt < tend;
      u4v* nxt = lds + (cur ^ 1) * BUFU;
      if (more) {   // the next chunk's loads, in flight during this chunk's products
        stage_load(g, st, nt, nc);
        weights_to_lds(g, nt, nc, nxt);
      }
      float inv = 1.f;
      chunk(lds + cur * BUFU, nxt, cb, rp, acc, st, more, inv);
      if (more && nc == 0) isx_next = inv;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the weight rows have landed
      __syncthreads();
      cur ^= 1;
    }
#if NFI_DCONV_EXP & 2
    {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) v += acc[i][j][r];
      if (v == 12345.f) g.y[threadIdx.x] = v;
    }
#else
    epilogue<EPI>(g, decode(g, t), cb, rp, acc, isx * w_inv, t);
#endif
    t += tstep;
    if (t >= tend) break;
  }
}

// w [Co][Ci][3][3] -> wp [2][9][Ci'/8][Co'][8] halves (hi, lo of w 2^e) and w_inv = 2^-e; flip: the
// data gradient's weight w'[ci][co][ky][kx] = w[co][ci][2 - ky][2 - kx] (Co' = Ci, Ci' = Co).  Three
// launches, once per frozen weight: max |w| into w_inv[0] (float bits, atomicMax, zeroed first), the
// pack (every block reads the maximum), then w_inv[0] = 2^-e.
__global__ void __launch_bounds__(256) wmax_kernel(const float* __restrict__ w, int n, unsigned* __restrict__ m) {
  float v = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) v = fmaxf(v, fabsf(w[i]));
  v = wave_max(v);
  if (lane_id() == 0) atomicMax(m, __float_as_uint(v));
}

__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ w, int Co, int Ci, int flip,
                                                   unsigned short* __restrict__ wp, const float* __restrict__ wmax) {
  const int n = Co * Ci * 9;
  float s, inv;
  pow2_scale15(wmax[0], s, inv);
  const int Cop = flip ? Ci : Co, Cip = flip ? Co : Ci;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256) {
    // q = ((tap Ci'/8 + ci' / 8) Co' + co') 8 + ci' % 8
    const int e = q & 7, u = q >> 3;
    const int co = u % Cop, rest = u / Cop;
    const int k8 = rest % (Cip / 8), tap = rest / (Cip / 8);
    const int ci = 8 * k8 + e;
    const float v = (flip ? w[((long long)ci * Ci + co) * 9 + (8 - tap)] : w[((long long)co * Ci + ci) * 9 + tap]) * s;
    const _Float16 h = (_Float16)v;
    wp[q] = __builtin_bit_cast(unsigned short, h);
    wp[n + q] = __builtin_bit_cast(unsigned short, (_Float16)(v - (float)h));
  }
}

__global__ void winv_kernel(float* w_inv) {
  float s, inv;
  pow2_scale15(w_inv[0], s, inv);
  w_inv[0] = inv;
}

// per-image max |x[n][c][p] s[n][c]| into the split slots (zeroed by the caller): grid (blocks, N)
__global__ void __launch_bounds__(256) absmax_scaled_kernel(const float* __restrict__ x, const float* __restrict__ sc,
                                                            int C, int HW, unsigned* __restrict__ slots) {
  const int n = blockIdx.y;
  const long long per = (long long)C * HW;
  const float4* x4 = reinterpret_cast<const float4*>(x + (long long)n * per);
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < per / 4; i += (long long)gridDim.x * 256) {
    const float4 v = x4[i];
    const float s = fabsf(sc[(long long)n * C + (int)(4 * i / HW)]);
    m = fmaxf(m, s * fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  m = wave_max(m);
  if (lane_id() == 0) atomicMax(slots + split_slot(n, blockIdx.x * 4 + (threadIdx.x >> 6)), __float_as_uint(m));
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

}  // namespace dconv
}  // namespace nfi

using namespace nfi;

extern "C" {

int32_t nfi_dconv_pack(const float* w, int32_t Co, int32_t Ci, int32_t flip, uint16_t* wp, float* w_inv, void* stream) {
  NFI_REQUIRE(w && wp && w_inv, "dconv_pack: null pointer");
  NFI_REQUIRE(Co > 0 && Ci > 0 && (flip ? Co : Ci) % 8 == 0 && (long long)Co * Ci * 9 < (1ll << 30),
              "dconv_pack: bad shape Co=%d Ci=%d (input channels of the packed form a multiple of 8)", Co, Ci);
  hipStream_t st = (hipStream_t)stream;
  NFI_REQUIRE(hipMemsetAsync(w_inv, 0, 4, st) == hipSuccess, "dconv_pack: memset");
  const int n = Co * Ci * 9, nb = std::min(1024, (n + 255) / 256);
  hipLaunchKernelGGL(dconv::wmax_kernel, dim3(nb), dim3(256), 0, st, w, n, reinterpret_cast<unsigned*>(w_inv));
  hipLaunchKernelGGL(dconv::pack_kernel, dim3(nb), dim3(256), 0, st, w, Co, Ci, flip ? 1 : 0,
                     reinterpret_cast<unsigned short*>(wp), w_inv);
  hipLaunchKernelGGL(dconv::winv_kernel, dim3(1), dim3(1), 0, st, w_inv);
  NFI_CHECK_LAUNCH("dconv pack_kernel");
  return NFI_OK;
}

int32_t nfi_absmax_scaled_slots(const float* x, const float* scale, int32_t N, int32_t C, int32_t HW, uint32_t* slots,
                                void* stream) {
  NFI_REQUIRE(x && scale && slots && N > 0 && N <= 65535 && C > 0 && HW > 0 && HW % 4 == 0 && ((uintptr_t)x & 15) == 0,
              "absmax_scaled_slots: bad arguments (HW %% 4 == 0, x 16-B aligned)");
  hipStream_t st = (hipStream_t)stream;
  NFI_REQUIRE(hipMemsetAsync(slots, 0, (SPLIT_SLOTS + 1) * 4, st) == hipSuccess, "absmax_scaled_slots: memset");
  const long long per4 = (long long)C * HW / 4;
  const int nb = (int)std::max<long long>(1, std::min<long long>((per4 + 255) / 256, std::max(1, 4096 / N)));
  hipLaunchKernelGGL(dconv::absmax_scaled_kernel, dim3((unsigned)nb, (unsigned)N), dim3(256), 0, st, x, scale, C, HW,
                     reinterpret_cast<unsigned*>(slots));
  NFI_CHECK_LAUNCH("absmax_scaled_kernel");
  return NFI_OK;
}

int32_t nfi_dconv3x3(const float* x, const float* xscale, const float* relu_y, const uint32_t* slots, const uint16_t* wp, const float* w_inv,
                     const float* bias, float* y, float* pooled, uint32_t* ymax, int32_t N, int32_t Ci, int32_t Co,
                     int32_t H, int32_t W, void* stream) {
  using namespace dconv;
  NFI_REQUIRE(x && slots && wp && w_inv && y, "dconv3x3: null pointer");
  NFI_REQUIRE(N > 0 && Ci > 0 && Ci % KC == 0 && Co > 0 && Co % CT == 0 && H > 0 && H % TR == 0 && W > 0 && W % TC == 0,
              "dconv3x3: bad shape N=%d Ci=%d Co=%d H=%d W=%d (Ci %% %d, Co %% %d, H %% %d, W %% %d must be 0)", N, Ci, Co,
              H, W, KC, CT, TR, TC);
  NFI_REQUIRE((long long)Ci * H * W * 4 < (1ll << 31) && (long long)2 * 9 * Ci * Co * 2 < (1ll << 31),
              "dconv3x3: an image or the weight past 2 GiB (32-bit buffer offsets)");
  NFI_REQUIRE(pooled == nullptr || bias != nullptr, "dconv3x3: pooling needs the bias/ReLU epilogue");
  NFI_REQUIRE(pooled == nullptr || relu_y == nullptr, "dconv3x3: the masked (data-gradient) form has no pool epilogue");
  NFI_REQUIRE(xscale == nullptr || (relu_y == nullptr && bias == nullptr),
              "dconv3x3: the scaled (modulated) form is a plain convolution (no mask, no epilogue)");
  NFI_REQUIRE(((uintptr_t)wp & 15) == 0, "dconv3x3: the packed weight must be 16-B aligned");
  Args g{x, relu_y, xscale, slots, reinterpret_cast<const u4v*>(wp), w_inv, bias, y, pooled, ymax, N, Ci, Co, H, W,
         W / TC, H / TR, Co / CT, 0};
  const long long T = (long long)N * g.th * g.tw * g.tco;
  NFI_REQUIRE(T < (1ll << 30), "dconv3x3: too many tiles");
  g.T = (int)T;
  const int cus = cu_count();
  int G = (int)std::min<long long>(T, cus);   // one workgroup per CU
  if (G >= 8) G &= ~7;
  const dim3 grid((unsigned)G), block(NT);
  if (xscale)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<false, 0, true>), grid, block, 0, (hipStream_t)stream, g);
  else if (relu_y && !bias)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<true, 0>), grid, block, 0, (hipStream_t)stream, g);
  else if (relu_y)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<true, 1>), grid, block, 0, (hipStream_t)stream, g);
  else if (!bias)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<false, 0>), grid, block, 0, (hipStream_t)stream, g);
  else if (!pooled)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<false, 1>), grid, block, 0, (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(dconv::dconv_kernel<false, 2>), grid, block, 0, (hipStream_t)stream, g);
  NFI_CHECK_LAUNCH("dconv_kernel");
  return NFI_OK;
}

}  // extern "C"
