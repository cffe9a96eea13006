// stereo_kernels.h -- launch interface of stereo.hip (host driver: orbgpu.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/orbgpu.h"
#include "orbgpu_internal.h"

namespace orbgpu {

struct StereoArgs {
    // pyramid level l of pair p: left image at lvl_base[l] + p * lvl_pair[l], right image at
    // lvl_base_r[l] + p * lvl_pair[l], row pitch lvl_pitch[l] (one extractor's batch: right =
    // left + one frame, pair = two frames; two extractors' single frames: p = 0)
    const uint8_t* lvl_base[kMaxLevels];
    const uint8_t* lvl_base_r[kMaxLevels];
    size_t lvl_pair[kMaxLevels];
    int lvl_pitch[kMaxLevels], lvl_w[kMaxLevels], lvl_h[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];  // mvScaleFactors, mvInvScaleFactors
    const orbgpu_keypoint* kps;  // extraction outputs: frame f at + f * cap
    const uint8_t* desc;
    const int* counts;
    int cap;
    float bf;      // mbf
    float max_d;   // mbf / mb (Frame.cpp:581)
    int th_orb;    // (TH_HIGH + TH_LOW) / 2
    int rr;        // rows scanned either side of vL: ceil(2 * max scale) + 1
    float* uright; // pair p: + p * cap
    float* depth;
    int* sad;      // scratch: accepted SAD per left keypoint or -1 (pair p: + p * cap)
};

size_t stereo_lds_bytes(int cap, int H);
hipError_t launch_stereo(const StereoArgs& a, int npairs, hipStream_t stream);

}  // namespace orbgpu
