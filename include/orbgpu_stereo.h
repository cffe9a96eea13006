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
 * d_uright / d_depth: float per left keypoint at + p * kp_capacity.
 * Calls on one extractor from different streams each get their own scratch. */
int orbgpu_stereo_matches_batch_device(orbgpu_extractor* ex, const uint8_t* d_images, size_t row_step,
                                       size_t frame_step, int npairs, const orbgpu_keypoint* d_kps,
                                       const uint8_t* d_desc, const int* d_counts, int kp_capacity,
                                       float bf, float min_z, float* d_uright, float* d_depth, void* stream);

/* The stereo Frame of the reference (Frame.cpp:66-127) extracts the left and
 * right images with two ORBextractor objects (two orbgpu_extractor handles of
 * the same geometry, one orbgpu_extract() call each) and then calls
 * ComputeStereoMatches: this is that call.  The pyramids are those of each
 * extractor's LAST orbgpu_extract() (read in place in HBM, never copied to
 * the host); kps / desc are the host outputs of those calls (n_l, n_r
 * keypoints).  Writes uright / depth[n_l] (-1 where unmatched).  Runs on the
 * calling thread's stream (host_ctx.h) and returns when the results are in
 * uright / depth. */
int orbgpu_stereo_matches_pair(orbgpu_extractor* left, orbgpu_extractor* right, const orbgpu_keypoint* kps_l,
                               const uint8_t* desc_l, int n_l, const orbgpu_keypoint* kps_r,
                               const uint8_t* desc_r, int n_r, float bf, float min_z, float* uright,
                               float* depth);

#ifdef __cplusplus
}
#endif
#endif
