/*
 * orbgpu_ransac.h -- C ABI of the RANSAC inner loops (Sim3Solver, PnPsolver)
 * and of the random stream that drives them.
 *
 * Reference (paths relative to /root/reference/ORB-SLAM2):
 *   DUtils::Random::RandomInt / SeedRand   Thirdparty/DBoW2/DUtils/Random.cpp:33-50
 *   Sim3Solver                              include/Sim3Solver.h:35-125, src/Sim3Solver.cpp:37-447
 *   PnPsolver                               include/PnPsolver.h:59-188, src/PnPsolver.cpp:104-1080
 *
 * The RANSAC loops of the reference draw their minimal sets with
 * DUtils::Random::RandomInt, i.e. with the process-wide glibc rand().  The
 * GPU evaluates many hypotheses at once, so the host must know the draws of
 * hypotheses that may never be used and must then consume exactly as many
 * draws as the sequential loop would have.  orbgpu_rand*() is a
 * bit-identical restatement of glibc's rand()/srand() (TYPE_3 additive
 * feedback generator) whose state can be saved and restored; a maintainer
 * routes DUtils::Random through it so every consumer of the
 * stream -- Initializer included -- sees the reference's sequence.
 *
 * Conventions as in orbgpu.h: int status returns, orbgpu_last_error().
 */
#ifndef ORBGPU_RANSAC_H
#define ORBGPU_RANSAC_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------- */
/* glibc-compatible random stream                                          */
/* ---------------------------------------------------------------------- */
typedef struct orbgpu_rand_state {
    int32_t r[31]; /* additive feedback table (glibc random_r TYPE_3) */
    int32_t f, b;  /* front / rear indices                              */
} orbgpu_rand_state;

/* srand(seed) / rand() of glibc on a process-wide state (thread-safe). */
void orbgpu_srand(unsigned int seed);
int orbgpu_rand(void);
/* DUtils::Random::RandomInt(min, max) = int(rand()/(RAND_MAX+1.0)*(max-min+1)) + min */
int orbgpu_random_int(int min, int max);
void orbgpu_rand_get_state(orbgpu_rand_state* out);
void orbgpu_rand_set_state(const orbgpu_rand_state* in);
/* explicit-state forms */
void orbgpu_srand_r(orbgpu_rand_state* st, unsigned int seed);
int orbgpu_rand_r(orbgpu_rand_state* st);

/* ---------------------------------------------------------------------- */
/* Sim3Solver RANSAC                                                        */
/* ---------------------------------------------------------------------- */
/* One solver (= one Sim3Solver object) of a batch.  Its correspondences
 * are points [offset, offset + n) of the batch arrays:
 *   X1, X2   float[3] per point: mvX3Dc1 / mvX3Dc2 (camera frames of KF1/KF2)
 *   maxerr1/2 float per point: (float)mvnMaxError1/2 -- the reference keeps
 *            9.210*sigma^2 in a vector<size_t>, i.e. truncated
 *            (Sim3Solver.cpp:92-93, Sim3Solver.h:78-79)
 * Hypothesis h of this call uses the correspondence triplet
 * samples[3*(sample_offset + h) .. +2] (indices into 0..n-1, already
 * resolved through the reference's swap-remove draw, Sim3Solver.cpp:174-183).
 * The call runs iterate()'s loop (Sim3Solver.cpp:147-221) over n_hyp
 * hypotheses: best update on inliers >= best_inliers, stop at the first
 * hypothesis with inliers > min_inliers. */
typedef struct orbgpu_sim3_problem {
    int n, offset;
    int fix_scale;       /* mbFixScale                                      */
    int min_inliers;     /* mRansacMinInliers                               */
    int best_inliers;    /* mnBestInliers before this call                  */
    int n_hyp;           /* hypotheses to run in this call                  */
    int sample_offset;   /* first triplet in samples[]                       */
    int pad;
    float K1[4], K2[4];  /* fx, fy, cx, cy of KF1 / KF2                      */
} orbgpu_sim3_problem;

typedef struct orbgpu_sim3_result {
    int found;           /* a hypothesis with inliers > min_inliers: iterate() returns T12 */
    int consumed;        /* hypotheses consumed (mnIterations advance)      */
    int best_inliers;    /* mnBestInliers after the call                    */
    int best_hyp;        /* hypothesis (0..n_hyp-1) that last updated the best, or -1 */
    float T12[16];       /* mBestT12 (row-major 4x4) when best_hyp >= 0     */
    float R12[9];        /* mBestRotation                                   */
    float t12[3];        /* mBestTranslation                                */
    float s12;           /* mBestScale                                      */
} orbgpu_sim3_result;

/* Device scratch for orbgpu_sim3_ransac_batch_device(): one hypothesis
 * record per sample triplet. */
size_t orbgpu_sim3_workspace_bytes(int total_samples);
/* Batched, HBM-resident (problems included): max_hyp >= every n_hyp;
 * d_workspace of orbgpu_sim3_workspace_bytes(total triplets); d_inliers
 * gets one byte per point (the inlier mask of best_hyp; untouched for a
 * problem whose best did not change).  Asynchronous on `stream`. */
int orbgpu_sim3_ransac_batch_device(int batch, const orbgpu_sim3_problem* d_problems, int max_hyp,
                                    const float* d_X1, const float* d_X2, const float* d_maxerr1,
                                    const float* d_maxerr2, const int* d_samples, void* d_workspace,
                                    orbgpu_sim3_result* d_results, uint8_t* d_inliers, void* stream);
/* Host-pointer form (uploads, runs, downloads, synchronises). */
int orbgpu_sim3_ransac_batch(int batch, const orbgpu_sim3_problem* problems, int total_points, const float* X1,
                             const float* X2, const float* maxerr1, const float* maxerr2, int total_samples,
                             const int* samples, orbgpu_sim3_result* results, uint8_t* inliers);

/* ---------------------------------------------------------------------- */
/* PnPsolver RANSAC (EPnP)                                                 */
/* ---------------------------------------------------------------------- */
/* One solver (= one PnPsolver object).  Correspondences [offset, offset+n):
 *   P3w   float[3] per point: mvP3Dw (world positions of the MapPoints)
 *   P2    float[2] per point: mvP2D (undistorted keypoints)
 *   maxerr float per point: mvMaxError = sigma^2 * th2 (PnPsolver.cpp:190-194)
 * Hypothesis h uses the 4-tuple samples[4*(sample_offset + h) .. +3]
 * (indices into 0..n-1 after the reference's swap-remove draw, :229-244);
 * sample ranges of different problems must not overlap.  The call replays
 * iterate()'s loop body (:224-299) over n_hyp hypotheses -- the caller
 * computes n_hyp from the reference's `||` loop condition (:224). */
typedef struct orbgpu_pnp_problem {
    int n, offset;
    int min_inliers;     /* mRansacMinInliers (after SetRansacParameters)   */
    int best_inliers;    /* mnBestInliers before this call                  */
    int n_hyp;           /* hypotheses to run in this call                  */
    int sample_offset;   /* first 4-tuple in samples[]                       */
    float fu, fv, uc, vc;
} orbgpu_pnp_problem;

typedef struct orbgpu_pnp_result {
    int found;           /* Refine() succeeded: iterate() returns mRefinedTcw */
    int consumed;        /* hypotheses consumed (mnIterations advance)      */
    int best_inliers;    /* mnBestInliers after the call                    */
    int best_hyp;        /* hypothesis that last became the best, or -1     */
    int refined_inliers; /* mnRefinedInliers when found                     */
    float best_Tcw[16];  /* mBestTcw when best_hyp >= 0 (row-major 4x4)     */
    float refined_Tcw[16]; /* mRefinedTcw when found                        */
} orbgpu_pnp_result;

/* Device scratch for orbgpu_pnp_ransac_batch_device(). */
size_t orbgpu_pnp_workspace_bytes(int total_points, int total_samples);
/* Batched, HBM-resident.  total_points / total_samples size the arrays and
 * the workspace (orbgpu_pnp_workspace_bytes); max_hyp >= every n_hyp.
 * d_best_mask (byte per point) is in/out: it must hold the incoming best
 * hypothesis' inliers (mvbBestInliers) when best_inliers > 0 and is
 * rewritten when the best changes; d_refined_mask gets mvbRefinedInliers of
 * the last Refine().  Asynchronous on `stream`. */
int orbgpu_pnp_ransac_batch_device(int batch, const orbgpu_pnp_problem* d_problems, int max_hyp,
                                   int total_points, int total_samples, const float* d_P3w, const float* d_P2,
                                   const float* d_maxerr, const int* d_samples, void* d_workspace,
                                   orbgpu_pnp_result* d_results, uint8_t* d_best_mask, uint8_t* d_refined_mask,
                                   void* stream);
/* Host-pointer form (uploads, runs, downloads, synchronises). */
int orbgpu_pnp_ransac_batch(int batch, const orbgpu_pnp_problem* problems, int total_points, const float* P3w,
                            const float* P2, const float* maxerr, int total_samples, const int* samples,
                            orbgpu_pnp_result* results, uint8_t* best_mask, uint8_t* refined_mask);

#ifdef __cplusplus
}
#endif
#endif
