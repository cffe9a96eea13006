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

// make `device` the calling thread's device for the host-form calls that follow
// (orbgpu_set_thread_device; device < 0: leave the thread's device alone)
inline void use_device(int device) {
    if (device >= 0 && orbgpu_set_thread_device(device) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
}

}  // namespace orbslam2_amd

#endif
