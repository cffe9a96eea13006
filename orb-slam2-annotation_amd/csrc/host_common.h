// host_common.h -- error reporting and device checks shared by the host
// translation units of liborbgpu.so (orbgpu.cpp, ransac.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/orbgpu.h"

namespace orbgpu {

// thread-local message returned by orbgpu_last_error()
extern thread_local std::string g_err;
int fail(int code, const std::string& msg);
// ORBGPU_OK when the current HIP device is a gfx950, else ORBGPU_ERR_NO_DEVICE
int check_device();

}  // namespace orbgpu

#define ORB_HIP(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return ::orbgpu::fail(ORBGPU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
