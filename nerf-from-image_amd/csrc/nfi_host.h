// Helpers shared by the C-ABI entry points (error reporting, launch checks) and the split-f16
// product's slot layout (used by its producers in three sources).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/nfi.h"

namespace nfi {
void set_error(const char* fmt, ...);
// Running-maximum slots of the split-f16 product's B operand (nfi_gemm.hip), PER IMAGE: image i's
// maximum of |B| lives in slots [i mod SPLIT_IMAGES][0..SPLIT_ISLOTS) (float bits, atomicMax'ed by
// its producer, spread over 64 slots per image as round 5's 64 shared slots were: producers' blocks
// run image by image, so fewer slots per image serialise their atomics — measured +0.14 ms per
// inversion step with 16), the completion counter at [SPLIT_SLOTS].  One power-of-two scale per
// image, so an image's operand precision never depends on the other images of its batch
// (include/nfi_producer.h).
constexpr int SPLIT_IMAGES = 256, SPLIT_ISLOTS = 64, SPLIT_SLOTS = SPLIT_IMAGES * SPLIT_ISLOTS;
__host__ __device__ __forceinline__ int split_slot(int img, int j) {
  return (img & (SPLIT_IMAGES - 1)) * SPLIT_ISLOTS + (j & (SPLIT_ISLOTS - 1));
}
}

#define NFI_REQUIRE(cond, ...)        \
  do {                                \
    if (!(cond)) {                    \
      nfi::set_error(__VA_ARGS__);    \
      return NFI_EINVAL;              \
    }                                 \
  } while (0)

#define NFI_CHECK_LAUNCH(what)                                                     \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      nfi::set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e_));    \
      return NFI_ELAUNCH;                                                          \
    }                                                                              \
  } while (0)
