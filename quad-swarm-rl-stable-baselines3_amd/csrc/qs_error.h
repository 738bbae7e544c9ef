// qs_error.h -- the library's last-error slot (qs_last_error), shared by its translation units.
#pragma once
#include <string>

#include <hip/hip_runtime.h>

// records msg as qs_last_error() and returns code (defined in qs_step.hip)
__attribute__((visibility("hidden"))) int qs_fail(int code, const std::string& msg);

#define QS_HIP_CHECK(call)                                                                              \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) return qs_fail(QS_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)
