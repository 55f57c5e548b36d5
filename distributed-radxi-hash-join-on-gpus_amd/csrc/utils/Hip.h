// HIP / RCCL error checking: every runtime call is checked and turned into an
// exception carrying rank and call site (SURVEY §5 "failure detection").
#pragma once

#include <hip/hip_runtime.h>

#include "Debug.h"

#define HIP_CHECK(expr)                                                                      \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      ::hpcjoin::utils::fail("HIP", __FILE__, __LINE__,                                      \
                             ::hpcjoin::utils::format("%s -> %s", #expr, hipGetErrorString(_e))); \
  } while (0)

#define HIP_CHECK_LAUNCH() HIP_CHECK(hipGetLastError())
