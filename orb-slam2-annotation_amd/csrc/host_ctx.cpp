// host_ctx.cpp -- the per-thread HostCtx of host_ctx.h.
#include "host_ctx.h"

#include <algorithm>
#include <memory>

namespace orbgpu {

HostCtx::~HostCtx() {
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
    static thread_local std::unique_ptr<HostCtx> t;
    if (!t) {
        auto c = std::make_unique<HostCtx>();
        ORB_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        t = std::move(c);
    }
    *out = t.get();
    return ORBGPU_OK;
}

}  // namespace orbgpu
