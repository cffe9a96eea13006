// proj_kernels.h -- launchers of proj.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/orbgpu_proj.h"

namespace orbgpu {

int proj_max_keypoints();
hipError_t launch_search_by_projection(int ncalls, const orbgpu_proj_call* calls, int stride, int* match,
                                       int* nmatches, hipStream_t stream);
hipError_t launch_is_in_frustum(const orbgpu_proj_target& T, int n, const float* pos, const float* normal,
                                const float* min_dist, const float* max_dist, float cos_limit, int* flags,
                                float* track, int* track_level, hipStream_t stream);

}  // namespace orbgpu
