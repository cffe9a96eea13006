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

/* ---------------------------------------------------------------------- */
/* Model hypotheses (Initialize / FindHomography / FindFundamental)        */
/* ---------------------------------------------------------------------- */
/* DUtils::Random::SeedRandOnce(seed) on the orbgpu_rand stream
 * (Thirdparty/DBoW2/DUtils/Random.cpp:38-45): seeds only on the first call
 * in the process, as Initialize's SeedRandOnce(0) (Initializer.cpp:102). */
void orbgpu_seed_rand_once(unsigned int seed);

/* Initialize's minimal sets (Initializer.cpp:96-115): for it < n_iter,
 * vAvailableIndices = 0..n_matches-1 and 8 x (RandomInt(0, size-1), swap
 * with back, pop) from the orbgpu_rand stream; sets[8*it + j] = mvSets[it][j]. */
int orbgpu_init_draw_sets(int n_matches, int n_iter, int* sets);

/* Workspace of orbgpu_init_hypotheses_batch_device (normalised points, T1, T2). */
size_t orbgpu_init_workspace_bytes(int n1, int n2);

/* Normalize (Initializer.cpp:965-1015) of mvKeys1 (d_kp1: n1 x (x, y)) and
 * mvKeys2 (d_kp2), then for every iteration it < n_iter the hypotheses of
 * FindHomography (:160-212: H21 = T2.inv()*ComputeH21(8 pairs)*T1, H12 =
 * H21.inv()) and FindFundamental (:217-269: F21 = T2.t()*ComputeF21*T1) from
 * the 8 matches d_sets[8 it ..] (indices into d_pairs: n_matches x (first,
 * second) = mvMatches12).  d_h21 / d_h12 / d_f21: n_iter x 9 row-major.
 * d_pts (nullable, 16-byte aligned): the n_matches orbgpu_match_pts the
 * scorers above read.  The 8-point SVDs are one-sided Jacobi in double --
 * the reference's cv::SVDecomp is not reproducible bit for bit -- so the
 * matrices equal the reference's to a tolerance (tests/test_init.py). */
int orbgpu_init_hypotheses_batch_device(const float* d_kp1, int n1, const float* d_kp2, int n2, const int* d_pairs,
                                        int n_matches, const int* d_sets, int n_iter, void* d_work,
                                        orbgpu_match_pts* d_pts, float* d_h21, float* d_h12, float* d_f21,
                                        void* stream);

/* FindHomography / FindFundamental's selection (Initializer.cpp:207-212,
 * :264-269): *best = the first h with scores[h] greater than every earlier
 * score and than 0; -1 when no score exceeds 0 (the reference keeps score 0
 * and an all-false inlier vector).  Host arrays. */
int orbgpu_init_select_best(const float* scores, int nhyp, int* best);

#ifdef __cplusplus
}
#endif
#endif
