// host_ctx.h -- per-thread staging for the host-form entry points: the calls
// the drop-in C++ classes (include/orbslam2_amd/*.h) make from the reference's
// Tracking, LocalMapping and LoopClosing threads (ORBmatcher, PnPsolver,
// Sim3Solver, Initializer, ORBVocabulary).
//
// Each thread gets one HostCtx on first use: a non-blocking HIP stream, a
// device arena and a pinned host mirror of the same capacity, grown
// geometrically and kept for the thread's lifetime.  A call (HostCall) lays
// its inputs and outputs out in the arena, packs the inputs into the pinned
// mirror, uploads them with ONE async copy, launches on the thread's stream,
// reads the outputs back with ONE async copy and waits on that stream only.
// No hipMalloc / hipFree / hipDeviceSynchronize per call, so the threads do
// not serialise against each other or against a batch stream.  The two copies
// are kernels (launch_copy16: reads or writes of the pinned mirror over PCIe)
// rather than copy-engine transfers, whose hand-off to and from the compute
// queue cost ~8 us each on the box (ORBGPU_HOST_ZEROCOPY=0: copy engine).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host_common.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

// transfers of the host-form calls by copy kernels (default) or the copy engine
inline bool host_copy_kernels() {
    static const bool v = [] {
        const char* s = std::getenv("ORBGPU_HOST_ZEROCOPY");
        return !(s && std::atoi(s) == 0);
    }();
    return v;
}

struct HostCtx {
    hipStream_t stream = nullptr;
    int device = -1;  // the HIP device the stream and arena belong to
    uint8_t* dev = nullptr;
    uint8_t* pin = nullptr;
    size_t cap = 0;
    ~HostCtx();
    int reserve(size_t bytes);  // device arena and pinned mirror >= bytes
};

// The calling thread's context (stream created on first use).
int host_ctx(HostCtx** out);

class HostCall {
  public:
    explicit HostCall(HostCtx& c) : c_(c) {}

    // Stage a call: `stage(*this)` is run twice, first to measure, then to
    // copy the inputs into the pinned mirror; the pointers in()/out() return
    // are device pointers in the arena (placeholders during the measuring
    // pass: stage must only store them).  Then one H2D copy of the region.
    template <class F>
    int run(F&& stage) {
        measuring_ = true;
        off_ = 0;
        stage(*this);
        const size_t total = off_;
        if (int rc = c_.reserve(total)) return rc;
        measuring_ = false;
        off_ = 0;
        stage(*this);
        used_ = off_;
        if (used_) {  // used_ is a multiple of 256 (take)
            if (host_copy_kernels())
                ORB_HIP(launch_copy16(c_.dev, c_.pin, used_, c_.stream));
            else
                ORB_HIP(hipMemcpyAsync(c_.dev, c_.pin, used_, hipMemcpyHostToDevice, c_.stream));
        }
        return ORBGPU_OK;
    }

    // inputs: a device copy of src[0..count) (nullptr for a null src)
    template <class T>
    T* in(const T* src, size_t count) {
        if (!src) return nullptr;
        const size_t o = take(count * sizeof(T));
        if (!measuring_ && count) std::memcpy(c_.pin + o, src, count * sizeof(T));
        return ptr<T>(o);
    }
    // outputs: uninitialised device space for count elements
    template <class T>
    T* out(size_t count) {
        return ptr<T>(take(count * sizeof(T)));
    }
    // outputs with initial contents (uploaded with the inputs); room for
    // max(count, room) elements
    template <class T>
    T* inout(const T* src, size_t count, size_t room = 0) {
        const size_t o = take((count > room ? count : room) * sizeof(T));
        if (!measuring_ && src && count) std::memcpy(c_.pin + o, src, count * sizeof(T));
        return ptr<T>(o);
    }

    // after the launches: read dptr[0..bytes) back into dst
    void fetch(const void* dptr, void* dst, size_t bytes) {
        if (!dptr || !dst || !bytes) return;
        const size_t o = static_cast<const uint8_t*>(dptr) - c_.dev;
        fetches_.push_back({o, bytes, dst});
    }
    // one D2H copy spanning every fetch, wait on the thread's stream, scatter
    int finish() {
        size_t lo = SIZE_MAX, hi = 0;
        for (auto& f : fetches_) {
            lo = f.off < lo ? f.off : lo;
            hi = f.off + f.bytes > hi ? f.off + f.bytes : hi;
        }
        if (hi > lo) {
            // the span widened to 16-byte bounds stays inside the arena (its slots are
            // 256-byte multiples); the extra bytes only overwrite staging copies
            const size_t lo16 = lo & ~size_t(15), hi16 = (hi + 15) & ~size_t(15);
            if (host_copy_kernels())
                ORB_HIP(launch_copy16(c_.pin + lo16, c_.dev + lo16, hi16 - lo16, c_.stream));
            else
                ORB_HIP(hipMemcpyAsync(c_.pin + lo, c_.dev + lo, hi - lo, hipMemcpyDeviceToHost, c_.stream));
        }
        ORB_HIP(hipStreamSynchronize(c_.stream));
        for (auto& f : fetches_) std::memcpy(f.dst, c_.pin + f.off, f.bytes);
        fetches_.clear();
        return ORBGPU_OK;
    }
    hipStream_t stream() const { return c_.stream; }

  private:
    struct Fetch {
        size_t off, bytes;
        void* dst;
    };
    size_t take(size_t bytes) {
        const size_t o = off_;
        off_ = (off_ + (bytes ? bytes : 4) + 255) & ~size_t(255);
        return o;
    }
    template <class T>
    T* ptr(size_t o) {
        // measuring pass: a non-null placeholder (the arena may move)
        return reinterpret_cast<T*>(measuring_ ? (uintptr_t)(o + 256) : (uintptr_t)(c_.dev + o));
    }
    HostCtx& c_;
    bool measuring_ = true;
    size_t off_ = 0, used_ = 0;
    std::vector<Fetch> fetches_;
};

}  // namespace orbgpu
