/*
 * orbgpu_init.h -- the scoring half of the monocular Initializer's two-model
 * RANSAC, batched over hypotheses on the GPU (conventions as orbgpu.h):
 *   Initializer::CheckHomography   src/Initializer.cpp:390-495
 *   Initializer::CheckFundamental  src/Initializer.cpp:497-594
 * FindHomography / FindFundamental (:160-290) call these once per RANSAC
 * iteration (mMaxIterations = 200) with the same N matches; here all the
 * iterations' hypotheses are scored in one launch, one workgroup per
 * hypothesis.  The per-hypothesis score is accumulated in the reference's
 * order (match 0's two terms, then match 1's, ...) in float, so scores and
 * inlier flags are bit-identical to the reference's loop.  Choosing the best
 * iteration (first strict maximum over score 0) is
 * orbgpu_init_select_best, the reference's `if(currentScore>score)`.
 * The 8-point solvers ComputeH21 / ComputeF21 (:292-388, cv::SVDecomp) stay
 * on the host.
 */
#ifndef ORBGPU_INIT_H
#define ORBGPU_INIT_H

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One match of mvMatches12: (u1, v1) = mvKeys1[first].pt,
 * (u2, v2) = mvKeys2[second].pt.  Device arrays of it must be 16-byte
 * aligned (the kernels load a match as one float4); ORBGPU_ERR_ARG if not. */
typedef struct orbgpu_match_pts {
    float u1, v1, u2, v2;
} orbgpu_match_pts;

/* Initializer::CheckHomography for `nhyp` hypotheses over the same `n`
 * matches: hypothesis h is d_h21[9h..9h+8] (H21, row-major) and
 * d_h12[9h..9h+8] (H12 = H21.inv()).  d_scores[h] = the returned score;
 * d_inliers[h*n + i] = vbMatchesInliers[i] (0/1).  sigma = mSigma. */
int orbgpu_init_check_homography_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_h21,
                                              const float* d_h12, int nhyp, float sigma, float* d_scores,
                                              uint8_t* d_inliers, void* stream);

/* Initializer::CheckFundamental for `nhyp` hypotheses d_f21[9h..9h+8]
 * (F21, row-major); outputs as above. */
int orbgpu_init_check_fundamental_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_f21, int nhyp,
                                               float sigma, float* d_scores, uint8_t* d_inliers, void* stream);

/* Both of the above in one launch (nh homography + nf fundamental
 * hypotheses side by side in one grid), as Initializer::Initialize runs the
 * two searches concurrently (Initializer.cpp:133-138). */
int orbgpu_init_check_both_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_h21, const float* d_h12,
                                        int nh, const float* d_f21, int nf, float sigma, float* d_scores_h,
                                        uint8_t* d_inliers_h, float* d_scores_f, uint8_t* d_inliers_f, void* stream);

/* FindHomography / FindFundamental's selection (Initializer.cpp:207-212,
 * :264-269): *best = the first h with scores[h] greater than every earlier
 * score and than 0; -1 when no score exceeds 0 (the reference keeps score 0
 * and an all-false inlier vector).  Host arrays. */
int orbgpu_init_select_best(const float* scores, int nhyp, int* best);

#ifdef __cplusplus
}
#endif
#endif
