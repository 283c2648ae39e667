// okm_hip_try.h — status plumbing shared by the library's HIP translation
// units: a failing HIP call or library step returns its okm_status (with the
// thread-local message set) from the enclosing function.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "okm_internal.h"

namespace okm {

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail(e_ == hipErrorOutOfMemory ? OKM_E_NOMEM : OKM_E_DEVICE,                  \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                      \
    } while (0)

#define OKM_TRY(expr)                    \
    do {                                 \
        okm_status s_ = (expr);          \
        if (s_ != OKM_OK) return s_;     \
    } while (0)

}  // namespace okm
