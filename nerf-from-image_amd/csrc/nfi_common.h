// nfi — MI355X-native volume renderer for the SDF-NeRF inversion loop of
// yuliangguo/nerf-from-image.  Shared device helpers (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nfi {

constexpr int WAVE = 64;
constexpr int NC = 32;     // tri-plane channels (generator.py:476-477)
constexpr int NH = 64;     // decoder hidden width (generator.py:293)
constexpr int NO = 11;     // decoder outputs: 1 distance + 10 attention logits (generator.py:380-385)
constexpr int NA = 10;     // attention values (palette rows)

// Exact-f32 decoder = per-lane MFMA operand tables for v_mfma_f32_16x16x4_f32 (lane l: A[l&15][l>>4],
// B[l>>4][l&15]; C/D: row 4(l>>4)+reg, col l&15), built by nfi_decoder_pack_n from the
// gain-scaled EqualizedLinear weights W1s [64,32], b1s [64], W2s [NOUT,64], b2s [NOUT]:
//   DT1 [hb][l][t]     W1s[16hb + (l&15)][8(l>>4) + t]          layer 1 A (t = 0..7)
//   DB1 [hb][l][r]     b1s[16hb + 4(l>>4) + r]                  layer 1 C init
//   DT2 [hb][l][r]     W2s[l&15][16hb + 4(l>>4) + r]            layer 2 A (rows >= 11 zero)
//   DT3 [hb][l][t]     W2s[4t + (l>>4)][16hb + (l&15)]          d hidden = W2s^T gy, A (t = 0..2)
//   DT4 [cb][hb][l][r] W1s[16hb + 4(l>>4) + r][16cb + (l&15)]   d x = W1s^T d z, A
//   DB2 [16]           b2s (zero padded)
//   DT1S, DB1S         DT1 and DB1 times log2(e) (the field backward's layer-1 recompute)
// The same layout for a decoder of NOUT outputs (NOB row blocks of 16; the d hidden product
// W2s^T dY^T runs over KT k-steps of 4 output rows, stored padded to KTP):
//   DT2 [ob][hb][l][r] W2s[16ob + (l&15)][16hb + 4(l>>4) + r]
//   DT3 [hb][l][t]     W2s[4t + (l>>4)][16hb + (l&15)]          (t < KTP; rows >= NOUT zero)
//   DB2 [16 NOB]       b2s
// NOUT = 33: 1 distance + 32 features for the view-direction mapper (--use_viewdir,
// generator.py:376-377) uses these exact-f32 tables; the inversion decoder (NOUT = 11: 1 distance +
// 10 attention logits, or 3 colour features zero padded) is packed as DecH below.
template <int NOUT>
struct DecL {
  static constexpr int NOB = (NOUT + 15) / 16;
  static constexpr int KT = (NOUT + 3) / 4;
  static constexpr int KTP = (KT + 3) / 4 * 4;
  static constexpr int DT1 = 0;
  static constexpr int DB1 = DT1 + 4 * 64 * 8;
  static constexpr int DT2 = DB1 + 4 * 64 * 4;
  static constexpr int DT3 = DT2 + NOB * 4 * 64 * 4;
  static constexpr int DT4 = DT3 + 4 * 64 * KTP;
  static constexpr int DB2 = DT4 + 2 * 4 * 64 * 4;
  // the field backward's layer-1 recompute: DT1 and DB1 times log2(e), so that sigmoid(z) =
  // 1 / (1 + 2^-z') needs no scaling multiply (nfi_render.hip mlp_backward_mfma)
  static constexpr int DT1S = DB2 + 16 * NOB;
  static constexpr int DB1S = DT1S + 4 * 64 * 8;
  static constexpr int SIZE = DB1S + 4 * 64 * 4;
};
// Split-f16 decoder tables (the inversion decoder, NOUT = 11): A operands of
// v_mfma_f32_16x16x32_f16 (lane l: A[l&15][8(l>>4) + j], j < 8; B[8(l>>4) + j][l&15]; C/D row
// 4(l>>4) + r, col l&15) holding each gain-scaled fp32 weight times a power of two 2^e as an fp16
// pair hi + lo (hi = f16(w 2^e), lo = f16(w 2^e - hi), both round-to-nearest): per lane 4 dwords of
// hi halves, then 4 dwords of lo halves.  Three products hi.hi + hi.lo + lo.hi per contraction give
// the fp32 result to the error of an fp32 dot product (DESIGN.md §3 "Decoder on the matrix cores").
// The hidden unit of K-step kb (32 units: blocks 2kb, 2kb + 1) at k = 8q + j is
//   hk(kb, q, j) = 16 (2kb + (j >> 2)) + 4q + (j & 3)
// — the order in which lane (., q) holds a layer-1 accumulator block, so the activations and their
// gradients feed the next product from registers.
//   H1  [hb 4][l][8]       W1s[16hb + (l&15)][8(l>>4) + j] 2^e1                layer 1 A
//   B1S [hb][l][r 4]       b1s[16hb + 4(l>>4) + r] log2(e)                       layer 1 bias (base 2)
//   H2  [kb 2][l][8]       W2s[l&15][hk(kb, l>>4, j)] ln2 2^e2 (rows >= 11 zero) layer 2 A (the
//                          hidden activations arrive as softplus / ln 2)
//   H3  [hb][l][4]         k = 8(l>>4) + j: hi of W2s[k][16hb + (l&15)] 2^e3 for k < 16, the lo of
//                          W2s[k - 16][..] for k >= 16 (outputs >= 11 zero)      d hidden A: one
//                          MFMA gives hi.hi + lo.hi against [dY hi; dY hi], one hi.lo + lo.lo
//                          against [dY lo; dY lo]
//   H4  [cb 2][kb 2][l][8] W1s[hk(kb, l>>4, j)][16cb + (l&15)] 2^e4             d x A
//   B2  [16]               b2s
//   SC  [16]               2^-e1 log2(e), 2^-e2, C3 = max_h sum_o |W2s[o][h]| 2^e3, 2^-(e3 + e4)
// e1, e2, e4 put the matrix's largest |weight| in [2^14, 2^15); e3 its largest in [2^6, 2^7), so the
// d hidden product (<= C3 max|dY 2^ey| with dY scaled to C3 max|dY 2^ey| in [2^13, 2^14)) stays in
// fp16 range.
struct DecH {
  static constexpr int H1 = 0;
  static constexpr int B1S = H1 + 4 * 64 * 8;
  static constexpr int H2 = B1S + 4 * 64 * 4;
  static constexpr int H3 = H2 + 2 * 64 * 8;
  static constexpr int H4 = H3 + 4 * 64 * 4;
  static constexpr int B2 = H4 + 2 * 2 * 64 * 8;
  static constexpr int SC = B2 + 16;
  static constexpr int SIZE = SC + 16;
};
static_assert(DecH::SIZE == 7200, "split decoder layout");

constexpr int NOV = 33;    // decoder outputs with the view-direction mapper
constexpr int NVF = 32;    // view-direction mapper features (generator.py:376-377, 398-399)
constexpr int DEC_SIZE = DecH::SIZE;           // 7,200 floats (the inversion decoder: split-f16 tables)

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// A wide (64- / 128-bit) LDS store whose data VGPRs no instruction rewrites for 2 wait states.
// Measured on MI355X ("Wide LDS stores"): ds_write_b128 / b64 whose data tuple the
// next 1-2 VALU instructions rewrote stored the NEW value in some lanes when the LDS pipe was
// backed up.  LLVM's hazard recognizer pads this hazard only for VMEM / FLAT stores wider than 8
// bytes (GCNHazardRecognizer::createsVALUHazard), not for DS stores.  The two scheduling barriers
// keep the compiler from moving any instruction between the store and the s_nop, so whatever
// reuses the data registers comes after the 2 wait states; the store itself stays a compiler
// instruction (counted in lgkmcnt).  scripts/isa_lint.py checks every wide DS store of the build.
// (The address escapes into an empty statement ahead of the store: with only the "memory" clobber, a
// store through a __restrict__ pointer the s_nop statement cannot see was moved past it and merged with
// the next store; with the address as an operand of the s_nop statement itself, the register that
// materialises it was written between the store and the nop.)
#ifndef NFI_LDS_GAP
#define NFI_LDS_GAP 1   // 0: plain stores (and round 3's 32-bit kept-alive rows): A/B builds only
#endif
template <class T>
__device__ __forceinline__ void lds_st(T* p, const T& v) {
#if !NFI_LDS_GAP
  *p = v;
  return;
#endif
  typedef __attribute__((address_space(3))) T* lds_ptr;
  const lds_ptr lp = (lds_ptr)p;
  asm volatile("" ::"v"(lp));
  *p = v;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// lds_st with a scheduling barrier ahead of the store as well: in a region holding the splits of
// several stores' data (nfi_gemm.hip's B operand), the scheduler otherwise hoisted a store above the
// next store's arithmetic, leaving its trailing s_nop ~90 instructions later and the freed data
// register rewritten at once (caught by scripts/isa_lint.py)
template <class T>
__device__ __forceinline__ void lds_st_fenced(T* p, const T& v) {
  __builtin_amdgcn_sched_barrier(0);
  lds_st(p, v);
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// DPP lane move whose lanes without a source (past the row / wave edge, or in a row outside
// ROWS) keep `fill` — the identity of the scan it feeds, so no lane test follows the move.
// Controls: row_shr:d 0x110+d, row_shl:d 0x100+d, wave_shr:1 0x138, wave_shl:1 0x130,
// row_bcast:15 0x142, row_bcast:31 0x143.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp_fill(float v, float fill) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(fill), __float_as_int(v), CTRL, ROWS, 0xF, false));
}
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_fill(double v, double fill) {
  const unsigned long long vi = (unsigned long long)__double_as_longlong(v);
  const unsigned long long fi = (unsigned long long)__double_as_longlong(fill);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)fi, (int)(unsigned)vi, CTRL, ROWS, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(fi >> 32), (int)(unsigned)(vi >> 32), CTRL, ROWS,
                                                            0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double readlane(double v, int l) {
  const unsigned long long vi = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)vi, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(vi >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Sum over the 64 lanes; result in every lane.  DPP inside rows of 16, then cross-row swaps.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]  (xor 1)
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]  (xor 2)
  v += dpp_mov<0x141>(v);   // row_half_mirror      (8-lane groups)
  v += dpp_mov<0x140>(v);   // row_mirror           (16-lane rows)
  v += __shfl_xor(v, 16);
  auto s = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(s[0]) + __int_as_float(s[1]);
}

__device__ __forceinline__ float wave_max(float v) {
  for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
// the same on DPP inside rows, then across rows (one ds_bpermute instead of six)
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  v = fmaxf(v, __shfl_xor(v, 16));
  auto s = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(s[0]), __int_as_float(s[1]));
}

// Inclusive prefix sum / product over lanes 0..63 (Hillis-Steele).
__device__ __forceinline__ float wave_incl_sum(float v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    float t = __shfl_up(v, d);
    if (l >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ float wave_incl_prod(float v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    float t = __shfl_up(v, d);
    if (l >= d) v *= t;
  }
  return v;
}

__device__ __forceinline__ float readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// torch.sign
__device__ __forceinline__ float tsign(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// Explicitly rounded fp32 ops (no FMA contraction): geometry that decides box-mask and texel
// membership is evaluated in exactly ATen's CPU rounding order (see DESIGN.md "bit-faithful
// geometry"), so a sample on the box surface is classified as the reference classifies it.
// (`#pragma clang fp contract(off)` keeps the instructions free of the `contract` flag, so the
// backend cannot fuse them into an FMA after inlining — __fmul_rn alone does not prevent it.)
__device__ __forceinline__ float fmul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float fadd(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float fsub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ __forceinline__ float fdiv(float a, float b) {
#pragma clang fp contract(off)
  return a / b;
}

// torch.lerp on CPU (ATen LerpKernel lerp_vec): |w| < 0.5 ? fma(w, e-s, s) : fma(w-1, e-s, e)
__device__ __forceinline__ float tlerp(float a, float b, float w) {
  const float d = fsub(b, a);
  return (fabsf(w) < 0.5f) ? fmaf(w, d, a) : fmaf(w - 1.f, d, b);
}

// torch.linspace(0, 1, steps) on CPU: step*idx below halfway, fma(-step, steps-1-idx, 1) above
__device__ __forceinline__ float tlinspace01(int idx, int steps) {
  if (steps == 1) return 0.f;
  const float step = 1.0f / (float)(steps - 1);
  const int halfway = steps / 2;
  return (idx < halfway) ? fmul(step, (float)idx) : fmaf(-step, (float)(steps - idx - 1), 1.0f);
}

// torch.linalg.vector_norm(x, 2) of a 3-vector on CPU: sqrt(fma(z,z, fma(y,y, x*x)))
__device__ __forceinline__ float tnorm3(float x, float y, float z) {
  return sqrtf(fmaf(z, z, fmaf(y, y, fmul(x, x))));
}

// Philox-4x32-10 counter-based RNG (Salmon et al. 2011) for randomize=True sampling.
__device__ __forceinline__ uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// One uniform [0,1) per (ray, sample, stream) triple.
__device__ __forceinline__ float rng_uniform(unsigned long long seed, unsigned long long offset,
                                             long long ray, int sample, int stream) {
  uint4 c = make_uint4((uint32_t)ray, (uint32_t)((unsigned long long)ray >> 32),
                       (uint32_t)sample | ((uint32_t)stream << 24), (uint32_t)offset);
  uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(offset >> 32));
  return u01(philox4x32(c, k).x);
}

// ---------------------------------------------------------------------------------------
// Phase timing for profiling builds (-DNFI_STAMPS, scripts/stamps.py): per-wave s_memtime
// deltas summed into nfi_stamp_acc[slot][phase] (slots spread the atomics).  Compiled out of
// the product library.
// ---------------------------------------------------------------------------------------
constexpr int STAMP_PHASES = 32, STAMP_SLOTS = 1024;
#ifdef NFI_STAMPS
extern __device__ unsigned long long nfi_stamp_acc[STAMP_SLOTS * STAMP_PHASES];
#define NFI_STAMP_INIT unsigned long long nfi_st_ = __builtin_readcyclecounter();
#define NFI_STAMP(id)                                                                        \
  {                                                                                          \
    const unsigned long long n_ = __builtin_readcyclecounter();                             \
    if (lane_id() == 0)                                                                      \
      atomicAdd(&nfi::nfi_stamp_acc[(blockIdx.x & (STAMP_SLOTS - 1)) * STAMP_PHASES + (id)], \
                n_ - nfi_st_);                                                               \
    nfi_st_ = n_;                                                                            \
  }
#define NFI_STAMP_PARAM , unsigned long long& nfi_st_
#define NFI_STAMP_ARG , nfi_st_
#else
#define NFI_STAMP_INIT
#define NFI_STAMP(id)
#define NFI_STAMP_PARAM
#define NFI_STAMP_ARG
#endif

}  // namespace nfi
