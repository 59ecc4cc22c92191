// Microbenchmark: LDS float accumulation throughput on gfx950 — ds_add_f32 vs plain
// ds_read/ds_write read-modify-write, 64 distinct consecutive dwords per wave-instruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int MODE, int WAVES_PER_TILE>
__global__ void __launch_bounds__(256) k(float* out, int iters, int stride) {
  __shared__ float acc[4 * 9248];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  float* A = acc + (WAVES_PER_TILE == 1 ? wv * 9248 / 4 : 0);
  for (int i = threadIdx.x; i < 4 * 9248; i += 256) acc[i] = 0.f;
  __syncthreads();
  unsigned idx = (wv * 97) % 280;
  float v = 1.0f + l;
  for (int it = 0; it < iters; ++it) {
    idx = (idx * 13 + stride) % 280;   // texel row start (wave-uniform)
    float* p = A + idx * 32 + l;       // 64 consecutive floats (two texels)
    if (MODE == 0) {
      atomicAdd(p, v);
    } else {
      *p = *p + v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[threadIdx.x + 7];
}

int main() {
  float* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 3; ++mode) {
      hipEventRecord(a);
      if (mode == 0) k<0, 0><<<blocks, 256>>>(out, iters, 7);
      if (mode == 1) k<1, 1><<<blocks, 256>>>(out, iters, 7);
      if (mode == 2) k<0, 1><<<blocks, 256>>>(out, iters, 7);
      hipEventRecord(b);
      CHECK(hipEventSynchronize(b));
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double ops = (double)blocks * 4 * iters;   // wave-instructions
      printf("mode %d (%s): %.3f ms, %.1f wave-ops/ns chip, %.1f cycles/op/CU @2.4GHz\n", mode,
             mode == 0 ? "ds_add_f32 shared tile" : mode == 1 ? "RMW private tile" : "ds_add_f32 private tile",
             ms, ops / (ms * 1e6), (ms * 1e6 * 2.4) / (ops / 256));
    }
  }
  return 0;
}
