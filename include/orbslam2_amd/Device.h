// Device.h -- GPU placement of the drop-in classes (no reference equivalent:
// the reference is CPU-only).  Every class takes an optional trailing `device`
// constructor argument (default -1: the calling thread's current device);
// with device >= 0 its calls run on that GPU, so a host can put the two
// extraction threads of a stereo Frame (src/Frame.cpp:84-87), several camera
// streams or the LoopClosing solvers on different GPUs without linking HIP.
#ifndef ORBSLAM2_AMD_DEVICE_H
#define ORBSLAM2_AMD_DEVICE_H

#include <stdexcept>
#include <string>

#include "../orbgpu.h"

namespace orbslam2_amd {

// Makes `device` the calling thread's device for the guard's scope (one
// member call) and restores the thread's previous device at its end, as the
// extractor entry points do inside the library (DeviceScope): an object placed
// on GPU k never moves the thread -- or the default (device = -1) objects the
// thread uses after it -- to GPU k.  device < 0: the thread's device is left
// alone (the default objects run wherever the thread's device is).
class DeviceGuard {
  public:
    explicit DeviceGuard(int device) {
        if (device < 0) return;
        int cur = -1;
        if (orbgpu_get_thread_device(&cur) != ORBGPU_OK) cur = -1;
        if (cur == device) return;
        if (orbgpu_set_thread_device(device) != ORBGPU_OK)
            throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
        prev_ = cur;
    }
    ~DeviceGuard() {
        if (prev_ >= 0) (void)orbgpu_set_thread_device(prev_);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;

  private:
    int prev_ = -1;
};

}  // namespace orbslam2_amd

#endif
