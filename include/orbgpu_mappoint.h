/*
 * orbgpu_mappoint.h -- C ABI of the two MapPoint updates run on every point
 * that is created or fused (LocalMapping.cpp:206-208 ProcessNewKeyFrame,
 * :570-572 CreateNewMapPoints, :676-679 SearchInNeighbors; Tracking.cpp:673-675,
 * :864-866, :1461-1462; LoopClosing.cpp:611, :646; Optimizer.cpp:259, :883,
 * :1198), batched over points:
 *
 *   MapPoint::ComputeDistinctiveDescriptors   src/MapPoint.cpp:302-380
 *   MapPoint::UpdateNormalAndDepth            src/MapPoint.cpp:414-457
 *
 * A point's observations are the entries of its std::map<KeyFrame*, size_t>
 * mObservations in map order, laid out as CSR: point p owns observations
 * obs_offsets[p] .. obs_offsets[p+1]-1.  The caller skips points that are
 * bad (both members return at once for them).
 */
#ifndef ORBGPU_MAPPOINT_H
#define ORBGPU_MAPPOINT_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ComputeDistinctiveDescriptors: the descriptors of the observations whose
 * keyframe is not bad (obs_valid[o] != 0; NULL: all), their pairwise
 * DescriptorDistance, per descriptor the element (N-1)/2 of its sorted
 * distances (self included), and the first descriptor with the smallest such
 * median.  Outputs per point: best[p] = the observation (0-based, within the
 * point's whole list) whose descriptor becomes mDescriptor, or -1 when no
 * valid observation remains (the reference keeps mDescriptor then);
 * best_median[p] (optional) = its median distance, -1 with best.
 * obs_desc: 32 bytes per observation (pKF->mDescriptors.row(idx)). */
int orbgpu_compute_distinctive_descriptors_batch_device(int n_points, const int* d_obs_offsets,
                                                        const uint8_t* d_obs_desc, const uint8_t* d_obs_valid,
                                                        int* d_best, int* d_best_median, void* stream);
/* Host form (host pointers). */
int orbgpu_compute_distinctive_descriptors(int n_points, const int* obs_offsets, const uint8_t* obs_desc,
                                           const uint8_t* obs_valid, int* best, int* best_median);

/* UpdateNormalAndDepth: over ALL observations (bad keyframes included, as
 * the reference), normal += (Pos - Ow_i) / cv::norm(Pos - Ow_i) in map order,
 * mNormalVector = normal / n; dist = cv::norm(Pos - refKF centre),
 * mfMaxDistance = dist * mvScaleFactors[octave of the refKF observation],
 * mfMinDistance = mfMaxDistance / mvScaleFactors[nLevels-1].  Points without
 * observations keep their outputs (the reference returns early).  OpenCV
 * conventions restated: cv::norm of a float 3-vector is the double square
 * root of a double sum of squares; `a + b / s` is cv::scaleAdd with the
 * float scale (float)(1/s), `a / n` convertTo with the float scale (float)(1/n). */
typedef struct orbgpu_normal_depth_batch {
    int n_points;
    const int* obs_offsets;       /* n_points + 1                                        */
    const float* obs_Ow;          /* 3 per observation: its keyframe's GetCameraCenter() */
    const float* pos;             /* 3 per point: mWorldPos                              */
    const float* ref_Ow;          /* 3 per point: mpRefKF->GetCameraCenter()             */
    const float* ref_level_scale; /* per point: mpRefKF->mvScaleFactors[octave]          */
    const float* ref_max_scale;   /* per point: mpRefKF->mvScaleFactors[nLevels - 1]     */
    float* normal;                /* out, 3 per point: mNormalVector                     */
    float* min_dist;              /* out, per point: mfMinDistance                       */
    float* max_dist;              /* out, per point: mfMaxDistance                       */
} orbgpu_normal_depth_batch;

/* Device form: every pointer of *b (a host struct) on the device. */
int orbgpu_update_normal_and_depth_batch_device(const orbgpu_normal_depth_batch* b, void* stream);
/* Host form (host pointers). */
int orbgpu_update_normal_and_depth(const orbgpu_normal_depth_batch* b);

#ifdef __cplusplus
}
#endif
#endif
