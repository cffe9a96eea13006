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
// ORBGPU_ERR_ARG for a negative ordinal or one >= the visible device count,
// ORBGPU_ERR_NO_DEVICE when no device is visible
int validate_device(int device);

// Makes `device` the calling thread's current HIP device for the scope and
// restores the previous one (device < 0: leaves the thread's device alone).
// Every entry point that takes an extractor runs under the extractor's device,
// so a handle created on GPU k works from any thread (orbgpu_extractor_create_on_device).
class DeviceScope {
  public:
    explicit DeviceScope(int device) {
        int cur = -1;
        if (device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != device && hipSetDevice(device) == hipSuccess)
            prev_ = cur;
    }
    ~DeviceScope() {
        if (prev_ >= 0) (void)hipSetDevice(prev_);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;

  private:
    int prev_ = -1;
};

}  // namespace orbgpu

#define ORB_HIP(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return ::orbgpu::fail(ORBGPU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
