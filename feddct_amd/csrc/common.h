// common.h — internal helpers shared by the libfedagg.so translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/fedagg.h"

namespace fa {
// thread-local last-error message (fa_last_error); returns code
int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace fa

#define FA_HIP_TRY(expr)                                                        \
  do {                                                                          \
    hipError_t e_ = (expr);                                                     \
    if (e_ != hipSuccess)                                                       \
      return fa::set_err(FA_E_HIP, "%s: %s", #expr, hipGetErrorString(e_));    \
  } while (0)
