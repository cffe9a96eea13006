/*
 * orbgpu_mapping.h -- C ABI of LocalMapping::CreateNewMapPoints' per-match
 * triangulation (src/LocalMapping.cpp:369-515): for every pair of matched
 * keypoints that ORBmatcher::SearchForTriangulation returned between the
 * current keyframe (kf1) and one neighbour (kf2), the parallax test, linear
 * triangulation (or KeyFrame::UnprojectStereo, src/KeyFrame.cpp:747-775), the
 * positive-depth, reprojection (chi-square 5.991 / 7.8) and scale-consistency
 * tests.  One result per match: the 3-D point and whether the reference
 * creates a MapPoint from it (the MapPoint construction and map insertion,
 * :517-541, stay with the caller, in match order).
 *
 * The linear triangulation's cv::SVD::compute (float Jacobi) is restated as
 * one-sided Jacobi in double; the rest follows the reference's float
 * expressions (tolerance in tests/test_mapping.py).
 */
#ifndef ORBGPU_MAPPING_H
#define ORBGPU_MAPPING_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The fields of a KeyFrame CreateNewMapPoints reads. */
typedef struct orbgpu_mapping_kf {
    float Tcw[12];                  /* [GetRotation() | GetTranslation()], row-major 3 x 4 */
    float Ow[3];                    /* GetCameraCenter()                                  */
    float fx, fy, cx, cy, invfx, invfy;
    float bf, b;                    /* mbf, mb                                            */
    int n;                          /* keypoints                                          */
    const orbgpu_keypoint* kps_un;  /* mvKeysUn                                           */
    const orbgpu_keypoint* kps;     /* mvKeys (UnprojectStereo reads the raw position)    */
    const float* u_right;           /* mvuRight (NULL: monocular, all -1)                 */
    const float* depth;             /* mvDepth  (NULL: monocular)                         */
    float scale_factors[16];        /* mvScaleFactors                                     */
    float level_sigma2[16];         /* mvLevelSigma2                                      */
} orbgpu_mapping_kf;

/* One neighbour pair of CreateNewMapPoints: kf1 = mpCurrentKeyFrame, kf2 =
 * pKF2, `pairs` = vMatchedIndices (n x (idx1, idx2)), scale_factor = kf1's
 * mfScaleFactor (ratioFactor = 1.5f * it).  Outputs per match: x3d (3
 * floats) and ok (1 = the reference creates a MapPoint at x3d). */
typedef struct orbgpu_mapping_job {
    orbgpu_mapping_kf kf1, kf2;
    float scale_factor;
    int n;
    const int* pairs;
    float* x3d;
    uint8_t* ok;
} orbgpu_mapping_job;

/* Batched: d_jobs and everything they point to on the device (one job per
 * neighbour keyframe, all in one launch). */
int orbgpu_triangulate_matches_batch_device(int njobs, const orbgpu_mapping_job* d_jobs, int max_n, void* stream);
/* Host form of one job (host pointers). */
int orbgpu_triangulate_matches(const orbgpu_mapping_job* job);

#ifdef __cplusplus
}
#endif
#endif
