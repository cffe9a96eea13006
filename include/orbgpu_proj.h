/*
 * orbgpu_proj.h -- C ABI of the projection matchers:
 *   Frame::isInFrustum                                   src/Frame.cpp:305-368
 *   ORBmatcher::SearchByProjection(F, vpMapPoints, th)   src/ORBmatcher.cpp:63-155   (LOCAL)
 *   ORBmatcher::SearchByProjection(KF, Scw, vpPoints,
 *                                  vpMatched, th)        src/ORBmatcher.cpp:352-470  (SIM3)
 *   ORBmatcher::SearchByProjection(F, LastF, th, bMono)  src/ORBmatcher.cpp:1506-1641 (LAST_FRAME)
 *   ORBmatcher::SearchByProjection(F, KF, sAlreadyFound,
 *                                  th, ORBdist)          src/ORBmatcher.cpp:1661-1790 (KEYFRAME)
 *   ORBmatcher::Fuse(KF, vpMapPoints, th)                src/ORBmatcher.cpp:962-1115  (FUSE)
 *   ORBmatcher::Fuse(KF, Scw, vpPoints, th, vpReplace)   src/ORBmatcher.cpp:1119-1249 (FUSE_SIM3)
 *   ORBmatcher::SearchBySim3(KF1, KF2, vpMatches12, s12, R12, t12, th)
 *                                                        src/ORBmatcher.cpp:1253-1491 (SIM3_DIR x 2
 *                                                        + the agreement check: orbgpu_search_by_sim3)
 * with Frame::GetFeaturesInArea / AssignFeaturesToGrid (src/Frame.cpp:241-259,
 * :379-443), MapPoint::PredictScale (src/MapPoint.cpp:481-508) and
 * RadiusByViewingCos (ORBmatcher.cpp:157-163).
 *
 * MapPoints are passed as structure-of-arrays over a point index; the
 * reference's pointer tests become flags.  Matching is sequential in the
 * reference (an assignment hides a keypoint from later points), and the GPU
 * keeps that order: one wave per call walks the points in order with its
 * lanes over the candidate keypoints.
 *
 * Fuse and SearchBySim3 have no such dependency inside the search: each
 * point's best keypoint depends only on the geometry and the descriptors.
 * Those variants return one result PER POINT; what the reference then does
 * with it (MapPoint::Replace, AddObservation, the agreement of the two
 * SearchBySim3 directions) stays with the caller, in the reference's order
 * (include/orbslam2_amd/ORBmatcher.h does exactly that).
 */
#ifndef ORBGPU_PROJ_H
#define ORBGPU_PROJ_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORBGPU_PROJ_LOCAL = 0,      /* SearchByProjection(F, vpMapPoints, th)          */
    ORBGPU_PROJ_SIM3 = 1,       /* SearchByProjection(KF, Scw, vpPoints, vpMatched) */
    ORBGPU_PROJ_LAST_FRAME = 2, /* SearchByProjection(F, LastF, th, bMono)          */
    ORBGPU_PROJ_KEYFRAME = 3,   /* SearchByProjection(F, KF, sAlreadyFound, th, d)  */
    /* per-point variants (the output row is indexed by point, see below) */
    ORBGPU_PROJ_FUSE = 4,       /* Fuse(pKF, vpMapPoints, th): target Tcw = the keyframe's pose,
                                   u_right = mvuRight (chi-square 7.8 / 5.99 test), points need
                                   pos, normal, min_dist, max_dist, desc                     */
    ORBGPU_PROJ_FUSE_SIM3 = 5,  /* Fuse(pKF, Scw, vpPoints, th, ...): target Tcw = Scw         */
    ORBGPU_PROJ_SIM3_DIR = 6    /* one direction of SearchBySim3: last_Tcw = the points' own
                                   keyframe pose [R1w|t1w], target Tcw = [sR21|t21], target
                                   fx..cy = pKF1's (the reference projects both ways with
                                   pKF1's intrinsics, ORBmatcher.cpp:1257-1260); points need
                                   pos, min_dist, max_dist, desc                            */
};

/* Point flags */
#define ORBGPU_PT_VALID 1      /* pointer set, !isBad(), not already found, (LAST_FRAME: !mvbOutlier) */
#define ORBGPU_PT_HAS_OBS 2    /* pMP->Observations() > 0                          */

/* The frame (or keyframe) being searched. */
typedef struct orbgpu_proj_target {
    int n;                          /* keypoints                                  */
    const orbgpu_keypoint* kps;     /* mvKeysUn                                   */
    const uint8_t* desc;            /* mDescriptors, n x 32                       */
    const float* u_right;           /* mvuRight (NULL = monocular, all -1)        */
    /* occupancy before the call, per keypoint (mvpMapPoints / vpMatched):
     * 0 = NULL, 1 = a MapPoint without observations, 2 = one with observations */
    const uint8_t* occupied;
    float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY            */
    float fx, fy, cx, cy, bf, b;    /* intrinsics, mbf, mb                        */
    int n_levels;                   /* mnScaleLevels                              */
    float log_scale_factor;         /* mfLogScaleFactor                           */
    float scale_factors[16];        /* mvScaleFactors                             */
    float Tcw[16];                  /* CurrentFrame.mTcw (LOCAL: unused; SIM3: Scw) */
} orbgpu_proj_target;

/* The points matched into the target (structure of arrays, index i). */
typedef struct orbgpu_proj_points {
    int n;
    const int* flags;               /* ORBGPU_PT_*                                 */
    const float* pos;               /* world position, 3 per point                 */
    const float* normal;            /* mean viewing direction (SIM3), 3 per point  */
    const uint8_t* desc;            /* MapPoint::GetDescriptor(), 32 per point     */
    const float* min_dist;          /* mfMinDistance (0.8f applied inside)         */
    const float* max_dist;          /* mfMaxDistance (1.2f applied inside)         */
    const int* octave;              /* LAST_FRAME: LastFrame.mvKeys[i].octave      */
    const float* angle;             /* LAST_FRAME/KEYFRAME: source keypoint angle  */
    /* LOCAL: the isInFrustum() results (mbTrackInView in flags bit 2) */
    const float* track;             /* 4 per point: mTrackProjX, mTrackProjY, mTrackProjXR, mTrackViewCos */
    const int* track_level;         /* mnTrackScaleLevel                           */
} orbgpu_proj_points;

#define ORBGPU_PT_IN_VIEW 4         /* LOCAL: mbTrackInView                         */

typedef struct orbgpu_proj_call {
    int variant;                    /* ORBGPU_PROJ_*                               */
    int check_ori;                  /* mbCheckOrientation (LAST_FRAME, KEYFRAME)    */
    float nnratio;                  /* mfNNratio (LOCAL)                            */
    float th;                       /* th                                           */
    int orb_dist;                   /* KEYFRAME: ORBdist                            */
    int mono;                       /* LAST_FRAME: bMono                            */
    float last_Tcw[16];             /* LAST_FRAME: LastFrame.mTcw                   */
    orbgpu_proj_target target;
    orbgpu_proj_points points;
} orbgpu_proj_call;

/* Frame::isInFrustum for n points against a frame pose: writes track[4*i..]
 * (projX, projY, projXR, viewCos), track_level[i] and sets/clears
 * ORBGPU_PT_IN_VIEW in flags[i] (device pointers). */
int orbgpu_is_in_frustum_device(const orbgpu_proj_target* target, int n, const float* d_pos, const float* d_normal,
                                const float* d_min_dist, const float* d_max_dist, float viewing_cos_limit,
                                int* d_flags, float* d_track, int* d_track_level, void* stream);

/* Batched projection matching; d_calls and everything they point to on the
 * device.  Call c writes d_match + c*stride, for variants 0..3 one int per
 * target keypoint:
 *   >= 0 : the point index assigned to that keypoint by this call
 *     -1 : untouched by this call
 *     -2 : set to NULL by the rotation-consistency cull (LAST_FRAME, KEYFRAME)
 * and d_nmatches[c] (the reference's return value; -1 if the target has
 * more than `stride` or 4096 keypoints -- rejected, never truncated).
 * For the per-point variants (FUSE, FUSE_SIM3, SIM3_DIR) one int per POINT:
 * the target keypoint with the smallest Hamming distance in the point's
 * window (first in GetFeaturesInArea order on ties) when that distance is
 * <= TH_LOW (Fuse) / TH_HIGH (SearchBySim3), else -1; d_nmatches[c] = the
 * number of such points (-1: more than `stride` points or 4096 keypoints).
 * Descriptor arrays (target.desc, points.desc) are read as 16-byte vectors:
 * their device addresses must be 16-byte aligned (hipMalloc's are). */
int orbgpu_search_by_projection_batch_device(int ncalls, const orbgpu_proj_call* d_calls, int stride, int* d_match,
                                             int* d_nmatches, void* stream);
/* Host form of one call: every pointer in *call is a host pointer; match
 * holds target.n ints (points.n for the per-point variants). */
int orbgpu_search_by_projection(const orbgpu_proj_call* call, int* match, int* nmatches);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 * (ORBmatcher.cpp:1253-1491): both directions in one launch, then the
 * agreement check.  kf1/kf2: Tcw = each keyframe's pose, mvKeysUn,
 * descriptors, bounds, scale pyramid (fx..cy are taken from kf1 for both
 * directions, as the reference does).  pts1/pts2: GetMapPointMatches() of
 * each keyframe, one entry per keypoint; flags VALID = non-NULL, !isBad() and
 * not already matched (vbAlreadyMatched1 / vbAlreadyMatched2, :1282-1296).
 * R12 row-major.  match12[i1] (kf1.n ints) = the KF2 keypoint whose MapPoint
 * becomes vpMatches12[i1], or -1; *nfound = the return value. */
typedef struct orbgpu_sim3_search {
    orbgpu_proj_target kf1, kf2;
    orbgpu_proj_points pts1, pts2;
    float s12;
    float R12[9];
    float t12[3];
    float th;
} orbgpu_sim3_search;
int orbgpu_search_by_sim3(const orbgpu_sim3_search* search, int* match12, int* nfound);

#ifdef __cplusplus
}
#endif
#endif
