// device_state.h -- per-device, process-wide one-time launch state.
//
// Kernel attributes (hipFuncSetAttribute's dynamic-LDS limit) and device
// properties (the CU count a launcher sizes its grid by) belong to a device,
// not to the process: a launcher that sets or reads them once keeps one slot
// per device ordinal, filled on the first launch on that device by whichever
// thread gets there first.  The reference's hosts call the matchers and the
// stereo Frame from several threads (src/Frame.cpp:84-87, src/Tracking.cpp:
// 141-149, LoopClosing beside Tracking), and a host may place those objects on
// different GPUs (orbgpu_set_thread_device, orbgpu_extractor_create_on_device):
// a process-wide or thread-local "done" flag would leave the second device
// without the attribute.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <mutex>

namespace orbgpu {

constexpr int kMaxDeviceSlots = 64;

// The calling thread's current HIP device, or -1 (none, or an ordinal above
// the slots).
inline int current_device_slot() {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDeviceSlots) return -1;
    return dev;
}

// f(device) run once per device; every later call on that device returns its
// result.
class PerDeviceOnce {
  public:
    template <class F>
    hipError_t get(F&& f) {
        const int d = current_device_slot();
        if (d < 0) return hipErrorInvalidDevice;
        std::call_once(flag_[d], [&] { err_[d] = f(d); });
        return err_[d];
    }

  private:
    std::once_flag flag_[kMaxDeviceSlots];
    hipError_t err_[kMaxDeviceSlots] = {};
};

// The multiprocessor (CU) count of the current device, read once per device
// (256 on MI355X; 256 if the query fails).
inline int current_device_cus() {
    static std::atomic<int> cus[kMaxDeviceSlots] = {};
    const int d = current_device_slot();
    if (d < 0) return 256;
    int n = cus[d].load(std::memory_order_relaxed);
    if (n > 0) return n;
    n = 256;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
    cus[d].store(n, std::memory_order_relaxed);
    return n;
}

// A kernel's dynamic-LDS limit that only grows (the need depends on the
// geometry of the call), per device: raised under a mutex when a launch needs
// more than the device's kernel has been granted.
class PerDeviceLdsLimit {
  public:
    hipError_t ensure(const void* fn, size_t bytes) {
        const int d = current_device_slot();
        if (d < 0) return hipErrorInvalidDevice;
        if (bytes <= set_[d].load(std::memory_order_acquire)) return hipSuccess;
        std::lock_guard<std::mutex> g(mu_);
        if (bytes <= set_[d].load(std::memory_order_relaxed)) return hipSuccess;
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e == hipSuccess) set_[d].store(bytes, std::memory_order_release);
        return e;
    }

  private:
    std::mutex mu_;
    std::atomic<size_t> set_[kMaxDeviceSlots] = {};
};

}  // namespace orbgpu
