/*
 * orbgpu_loop.h -- C ABI of LoopClosing::ComputeSim3's hot loop: the
 * Sim3Solver set-up for every loop candidate that SearchByBoW(KF, KF) matched
 * well enough, and the round-robin RANSAC over all candidates of a query.
 *
 * Reference (paths relative to /root/reference/ORB-SLAM2):
 *   LoopClosing::ComputeSim3            src/LoopClosing.cpp:273-420
 *     SearchByBoW(mpCurrentKF, pKF)     :311 (orbgpu_search_by_bow_batch_device, orbgpu_bow.h)
 *     nmatches < 20 -> discarded        :314-318
 *     Sim3Solver(..); SetRansacParameters(0.99, 20, 300)   :322-324
 *     while (nCandidates > 0 && !bMatch) for each candidate: iterate(5) :339-356
 *   Sim3Solver::Sim3Solver              src/Sim3Solver.cpp:37-107
 *   Sim3Solver::SetRansacParameters     src/Sim3Solver.cpp:111-141
 *   Sim3Solver::iterate                 src/Sim3Solver.cpp:147-221
 *
 * Scope of the round-robin call.  After a candidate's iterate() returns a
 * Sim3 the reference runs SearchBySim3 + OptimizeSim3 (:358-392, outside the
 * hot path) and stops at the first candidate whose optimisation keeps >= 20
 * inliers.  Here that verification is taken to pass, so a query ends at the
 * first RANSAC success in the reference's candidate order -- the result the
 * caller then verifies.  Everything up to that point is the reference's:
 * the same candidates discarded, the same hypotheses drawn from the same
 * glibc rand() stream in the same order (iterate(5) per candidate per round),
 * the same acceptance.
 *
 * Random stream.  DUtils::Random is process-global, so the draws of a query
 * start where the caller's stream stands: each query carries the
 * orbgpu_rand_state to start from (orbgpu_rand_get_state() for a live
 * process, orbgpu_srand_r(seed) for a seeded one) and returns the state after
 * exactly the draws the reference consumed.  A batch of queries is a batch
 * of independent ComputeSim3 calls, each from its own state.
 *
 * Conventions as in orbgpu.h: int status returns, orbgpu_last_error();
 * *_device functions take HBM pointers and are asynchronous on `stream`.
 */
#ifndef ORBGPU_LOOP_H
#define ORBGPU_LOOP_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"
#include "orbgpu_ransac.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The keyframe data a Sim3Solver constructor reads (Sim3Solver.cpp:37-107).
 * All pointers are device pointers; slot i of the keyframe is keypoint i
 * and its MapPoint. */
typedef struct orbgpu_loop_keyframe {
    int n;                    /* keypoints = MapPoint slots (mvpMapPoints.size()) */
    int pad;
    float Rcw[9];             /* GetRotation(), row-major                        */
    float tcw[3];             /* GetTranslation()                                */
    float K[4];               /* fx, fy, cx, cy of mK                            */
    const float* mp_world;    /* n x 3: GetWorldPos() of MapPoint i              */
    const uint8_t* mp_valid;  /* MapPoint i exists and !isBad()                  */
    const int* octave;        /* mvKeysUn[i].octave                              */
    const float* sigma2;      /* mvLevelSigma2[octave]                           */
} orbgpu_loop_keyframe;

/* One Sim3Solver(pKF1 = kf1, pKF2 = kf2, vpMatched12, bFixScale).
 * vpMatched12 comes from SearchByBoW(KF1, KF2): d_match12 + c*match_stride
 * holds, per KF1 slot, the matched KF2 slot or -1; d_nmatches[c] is
 * SearchByBoW's return value. */
typedef struct orbgpu_sim3_candidate {
    int kf1, kf2;             /* indices into the keyframe table                 */
} orbgpu_sim3_candidate;

/* Device workspace of orbgpu_sim3_setup_batch_device: per candidate up to
 * match_stride correspondences (X1, X2, max errors, KF1 slot, and their image
 * projections mvP1im1 / mvP2im2).  Query it: the layout is the library's. */
size_t orbgpu_sim3_setup_workspace_bytes(int n_cand, int match_stride);

/* Sim3Solver constructors for n_cand candidates: for i1 ascending with
 * vpMatched12[i1] and both MapPoints valid, mvX3Dc1 = Rcw1*X3D1w + tcw1,
 * mvX3Dc2 likewise, mvnMaxError = (size_t)(9.210*sigma^2) (kept as float),
 * mvnIndices1 = i1, mvP1im1 / mvP2im2 = FromCameraToImage (:54-99).  d_n_corr[c] = N (mvpMapPoints1.size()).
 * Candidates with d_nmatches[c] < min_matches get N = -1 (discarded before
 * a solver is built, LoopClosing.cpp:314-318).  The workspace keeps the
 * correspondences for orbgpu_compute_sim3_batch_device. */
int orbgpu_sim3_setup_batch_device(int n_cand, const orbgpu_sim3_candidate* d_cands,
                                   const orbgpu_loop_keyframe* d_kfs, const int* d_match12, int match_stride,
                                   const int* d_nmatches, int min_matches, void* d_workspace, int* d_n_corr,
                                   void* stream);

/* One ComputeSim3 call: candidates [first_cand, first_cand + n_cand) of the
 * candidate table, in the reference's candidate order. */
typedef struct orbgpu_compute_sim3_query {
    int first_cand, n_cand;   /* n_cand <= ORBGPU_LOOP_MAX_CANDIDATES            */
    orbgpu_rand_state rng;    /* DUtils::Random state when the query starts      */
} orbgpu_compute_sim3_query;

#define ORBGPU_LOOP_MAX_CANDIDATES 64

typedef struct orbgpu_sim3_ransac_params {
    double probability;       /* 0.99 (LoopClosing.cpp:324)                      */
    int min_inliers;          /* 20                                              */
    int max_iterations;       /* 300                                             */
    int iterations_per_call;  /* 5: iterate(5, ...) (:346)                       */
    int fix_scale;            /* mbFixScale (stereo / RGB-D)                      */
} orbgpu_sim3_ransac_params;

typedef struct orbgpu_compute_sim3_result {
    int matched;              /* candidate (0..n_cand-1) whose iterate() returned a Sim3 first, or -1 */
    int round;                /* round of iterate() calls in which it returned  */
    int n_inliers;            /* nInliers of that iterate() call                */
    int hypotheses;           /* RANSAC iterations run by all candidates        */
    int draws;                /* rand() values consumed (3 per iteration)       */
    int pad;
    float T12[16];            /* the returned Scm (row-major 4x4 [sR t; 0 1])    */
    float R12[9];             /* GetEstimatedRotation()                          */
    float t12[3];             /* GetEstimatedTranslation()                       */
    float s12;                /* GetEstimatedScale()                             */
    orbgpu_rand_state rng_after; /* stream state after the query's draws       */
} orbgpu_compute_sim3_result;

/* Per candidate after the query: the solver's state. */
typedef struct orbgpu_sim3_candidate_state {
    int n;                    /* N correspondences (-1: discarded before RANSAC) */
    int max_iterations;       /* mRansacMaxIts after SetRansacParameters         */
    int iterations;           /* mnIterations consumed                           */
    int best_inliers;         /* mnBestInliers                                   */
    int discarded;            /* vbDiscarded at the end                          */
    int pad;
} orbgpu_sim3_candidate_state;

/* The while/for loop of ComputeSim3 (:339-356) for every query, one
 * workgroup per query.  Needs the workspace filled by
 * orbgpu_sim3_setup_batch_device for the same candidate table (n_cand
 * entries; every query's range must lie inside it).  d_inliers
 * (n_cand_total * match_stride bytes): for the matched candidate, its
 * correspondence inlier flags (mvbBestInliers; map through the KF1 slots of
 * orbgpu_sim3_corr_kf1_slots to get vbInliers). */
int orbgpu_compute_sim3_batch_device(int n_queries, const orbgpu_compute_sim3_query* d_queries,
                                     int n_cand, const orbgpu_sim3_candidate* d_cands, const orbgpu_loop_keyframe* d_kfs,
                                     int match_stride, const void* d_workspace, const int* d_n_corr,
                                     orbgpu_sim3_ransac_params params, orbgpu_compute_sim3_result* d_results,
                                     orbgpu_sim3_candidate_state* d_cand_states, uint8_t* d_inliers,
                                     void* stream);

/* Device pointer to candidate c's KF1 slots (mvnIndices1) inside the
 * workspace: int[match_stride], the first d_n_corr[c] valid. */
const int* orbgpu_sim3_corr_kf1_slots(const void* d_workspace, int n_cand, int match_stride, int c);

#ifdef __cplusplus
}
#endif
#endif
