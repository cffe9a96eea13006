// host_ctx.cpp -- the per-thread HostCtx of host_ctx.h.
#include "host_ctx.h"

#include <algorithm>
#include <memory>

namespace orbgpu {

HostCtx::~HostCtx() {
    DeviceScope ds(device);
    // errors are ignored: at process exit the runtime may already be gone
    if (stream) (void)hipStreamSynchronize(stream);
    if (dev) (void)hipFree(dev);
    if (pin) (void)hipHostFree(pin);
    if (stream) (void)hipStreamDestroy(stream);
}

int HostCtx::reserve(size_t bytes) {
    if (bytes <= cap) return ORBGPU_OK;
    const size_t ncap = std::max<size_t>({bytes, 2 * cap, size_t(4) << 20});
    ORB_HIP(hipStreamSynchronize(stream));
    if (dev) (void)hipFree(dev);
    if (pin) (void)hipHostFree(pin);
    dev = nullptr;
    pin = nullptr;
    cap = 0;
    ORB_HIP(hipMalloc((void**)&dev, ncap));
    ORB_HIP(hipHostMalloc((void**)&pin, ncap, hipHostMallocDefault));
    cap = ncap;
    return ORBGPU_OK;
}

int host_ctx(HostCtx** out) {
    // one context per (thread, device): the thread's current device -- the one
    // orbgpu_set_thread_device chose -- owns the stream, arena and mirror
    constexpr int kMaxDevices = 64;
    static thread_local std::unique_ptr<HostCtx> t[kMaxDevices];
    int dev = 0;
    ORB_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices) return fail(ORBGPU_ERR_UNSUPPORTED, "device ordinal above 63");
    std::unique_ptr<HostCtx>& c = t[dev];
    if (!c) {
        auto n = std::make_unique<HostCtx>();
        n->device = dev;
        ORB_HIP(hipStreamCreateWithFlags(&n->stream, hipStreamNonBlocking));
        c = std::move(n);
    }
    *out = c.get();
    return ORBGPU_OK;
}

}  // namespace orbgpu
