// Host-side helpers shared by the C-ABI entry points (error reporting, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/nfi.h"

namespace nfi {
void set_error(const char* fmt, ...);
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
