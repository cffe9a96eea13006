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
 * The model hypotheses (Normalize, ComputeH21 / ComputeF21) and the motion
 * recovery (ReconstructH / ReconstructF) are declared further below.
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

/* ---------------------------------------------------------------------- */
/* Motion and structure (ReconstructH / ReconstructF)                      */
/* ---------------------------------------------------------------------- */
#define ORBGPU_INIT_MODEL_H 0
#define ORBGPU_INIT_MODEL_F 1

typedef struct orbgpu_init_reconstruction {
    int ok;             /* the reference's return value                              */
    int best;           /* the hypothesis the decision looked at, or -1              */
    int n_hyp;          /* 8 (H), 4 (F), 0 when ReconstructH stops at d1/d2, d2/d3   */
    int n_good[8];      /* CheckRT's nGood per hypothesis                            */
    float parallax[8];  /* CheckRT's parallax (degrees) per hypothesis               */
    float R21[9];       /* hypothesis `best`: rotation (row-major) ...               */
    float t21[3];       /* ... and unit translation                                  */
} orbgpu_init_reconstruction;

/* Initializer::ReconstructH (model H, M21 = H21) / ReconstructF (model F,
 * M21 = F21) (src/Initializer.cpp:596-963) with CheckRT (:1017-1118),
 * Triangulate and DecomposeE: the 8 / 4 motion hypotheses on the host,
 * CheckRT of every hypothesis over every inlier match on the GPU (one block
 * per hypothesis), then the reference's choice.  kp1 / kp2: n1 / n2 x (x, y)
 * (mvKeys1 / mvKeys2), pairs: n_matches x (first, second) = mvMatches12,
 * inliers: vbMatchesInliers (0/1), K row-major, sigma = mSigma.  Host
 * arrays.  p3d (n1 x 3) and triangulated (n1) receive vP3D and
 * vbTriangulated when out->ok (zeros otherwise).  n_matches <= 16384.
 * The SVDs are Jacobi in double (OpenCV's float Jacobi is not reproducible):
 * equal to the reference within the tolerance of tests/test_init.py. */
int orbgpu_init_reconstruct(int model, const float* kp1, int n1, const float* kp2, int n2, const int* pairs,
                            int n_matches, const unsigned char* inliers, const float* M21, const float* K,
                            float sigma, float min_parallax, int min_triangulated, orbgpu_init_reconstruction* out,
                            float* p3d, unsigned char* triangulated);

/* Initializer::Initialize (src/Initializer.cpp:55-157) in one host call:
 * mvMatches12 from matches12 (n1 ints, -1 = unmatched), SeedRandOnce(0) and
 * the `iterations` minimal sets from the orbgpu_rand stream, every H / F
 * hypothesis and its score on the GPU, the kept iterations, RH = SH/(SH+SF)
 * and ReconstructH (RH > 0.40) or ReconstructF with minParallax 1.0 and
 * minTriangulated 50.  kp1 = the reference frame's mvKeysUn (n1 x (x, y)),
 * kp2 = the current frame's.  `out` as orbgpu_init_reconstruct; *rh = RH,
 * *model = the model reconstructed.  p3d / triangulated: n1 entries. */
int orbgpu_init_initialize(const float* kp1, int n1, const float* kp2, int n2, const int* matches12, const float* K,
                           float sigma, int iterations, orbgpu_init_reconstruction* out, float* rh, int* model,
                           float* p3d, unsigned char* triangulated);

#ifdef __cplusplus
}
#endif
#endif
