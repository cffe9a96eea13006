/*
 * orbgpu_stereo.h -- stereo matching of the MI355X-native ORB-SLAM2 front end.
 *
 * Replaces Frame::ComputeStereoMatches (src/Frame.cpp:540-748, declared in
 * include/Frame.h:121) for rectified stereo pairs: for every left keypoint,
 * the best right keypoint in its row band by descriptor distance, refined by
 * an 11x11 SAD search over +-5 px on the keypoint's pyramid level, a parabola
 * fit, and the median-based outlier cut.  Outputs are mvuRight and mvDepth
 * (-1 where unmatched).  Conventions as orbgpu.h.
 */
#ifndef ORBGPU_STEREO_H
#define ORBGPU_STEREO_H

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Pairs p = 0..npairs-1 are frames (2p, 2p+1) = (left, right) of the LAST
 * orbgpu_extract_batch_device() call on `ex` (its pyramid must still be in
 * place: call on the same stream before the next extraction), with the same
 * d_images / row_step / frame_step and the keypoint, descriptor and count
 * arrays that call wrote (kp_capacity as passed to it).  bf = mbf (baseline
 * x fx); min_z = Frame::mb at the time the reference calls
 * ComputeStereoMatches -- 0 in the reference's stereo constructor
 * (Frame.cpp:67, :98), which makes the maximum disparity infinite.
 * d_uright / d_depth: float per left keypoint at + p * kp_capacity. */
int orbgpu_stereo_matches_batch_device(orbgpu_extractor* ex, const uint8_t* d_images, size_t row_step,
                                       size_t frame_step, int npairs, const orbgpu_keypoint* d_kps,
                                       const uint8_t* d_desc, const int* d_counts, int kp_capacity,
                                       float bf, float min_z, float* d_uright, float* d_depth, void* stream);

#ifdef __cplusplus
}
#endif
#endif
