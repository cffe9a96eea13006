/*
 * orbref.h -- CPU restatement of ORB-SLAM2's front-end hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, the smoke
 * check in __graft_entry__.py and bench.py's cpu_baseline leg are the only
 * callers.  The product (liborbgpu.so) never links or calls it.
 *
 * PARITY STATUS: unpinned against a real OpenCV-2.4 build.  The reference
 * (SFXiang/ORB-SLAM2-Annotation) ships no tests, golden vectors or fixtures
 * for this path, and its ORBextractor.cpp cannot be compiled here (OpenCV
 * 2.4 is absent; writing header stand-ins for it is not allowed).  The
 * OpenCV-2.4 primitive arithmetic restated here (resize INTER_LINEAR,
 * GaussianBlur 7x7, FAST-9/16, fastAtan2, cvRound) is written down in
 * DESIGN.md section "Spec decisions".  glibc sinf/cosf IS pinned: the
 * restatement matches the host libm bit-for-bit on every float in [0, 6.3]
 * (tools/check_sincosf.c).
 *
 * All functions are plain C ABI so tests can load liborbref.so via ctypes.
 */
#ifndef ORBREF_H
#define ORBREF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as cv::KeyPoint (OpenCV 2.4): pt.x, pt.y, size, angle,
 * response, octave, class_id -- 28 bytes. */
typedef struct orbref_kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbref_kp;

typedef struct orbref_extractor orbref_extractor;

/* ORBextractor::ORBextractor  (ORBextractor.cpp:412-472) */
orbref_extractor* orbref_create(int nfeatures, float scale_factor, int nlevels,
                                int ini_th_fast, int min_th_fast);
void orbref_destroy(orbref_extractor* ex);
/* DistributeOctTree tie-break among equal-size nodes: 0 = creation sequence
 * (the spec, default), 1 = reversed sequence, 2 = heap address of the
 * oracle's own list node, 3 = heap address under the REFERENCE'S allocation
 * pattern (octree_faithful.h: ExtractorNode layout, reserve / copy / erase
 * sequence) in this process's glibc heap, 4 = the same after a heap
 * perturbation, 5 = the same pattern under a deterministic glibc model.  For
 * the H2 measurement only (tools/h2_tiebreak.py); process-global. */
void orbref_set_tiebreak(int mode);

/* ORBextractor::operator()  (ORBextractor.cpp:1053-1117).
 * Returns the number of keypoints written (>= 0), or -1 if `capacity` is too
 * small (nothing is written then).  desc: n x 32 bytes. */
int orbref_extract(orbref_extractor* ex, const uint8_t* img, int width, int height,
                   size_t step, orbref_kp* kps, uint8_t* desc, int capacity);

/* Accessors for the state the last orbref_extract() left behind. */
int orbref_level_count(const orbref_extractor* ex);
int orbref_level_size(const orbref_extractor* ex, int level, int* w, int* h);
/* level `level` of mvImagePyramid in place (tight rows, step = w) */
const uint8_t* orbref_level_ptr(const orbref_extractor* ex, int level, int* w, int* h);
/* copies level `level` of mvImagePyramid (tight rows, w*h bytes) */
int orbref_level_copy(const orbref_extractor* ex, int level, uint8_t* dst);
/* FAST candidates of a level in vToDistributeKeys order, coordinates
 * relative to (minBorderX, minBorderY) = (16, 16): returns count, writes up
 * to cap entries of (x, y, score). */
int orbref_level_candidates(const orbref_extractor* ex, int level, int* xys, int cap);
/* keypoints kept by DistributeOctTree for a level, in list order, before the
 * +16 border shift: (x, y, score) */
int orbref_level_octree(const orbref_extractor* ex, int level, int* xys, int cap);
int orbref_features_per_level(const orbref_extractor* ex, int* out);
void orbref_scale_factors(const orbref_extractor* ex, float* scale, float* inv_scale,
                          float* sigma2, float* inv_sigma2);

/* --- primitives (OpenCV 2.4 semantics as restated in DESIGN.md) --- */
void orbref_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstep,
                             uint8_t* dst, int dw, int dh, size_t dstep);
void orbref_gaussian7_u8(const uint8_t* src, int w, int h, size_t sstep,
                         uint8_t* dst, size_t dstep);
/* cv::FAST(img, kps, threshold, nonmax=true), TYPE_9_16; writes (x, y, score)
 * row-major; returns count (or -1 when cap exceeded). */
int orbref_fast(const uint8_t* img, int w, int h, size_t step, int threshold,
                int* xys, int cap);
float orbref_fast_atan2(float y, float x);
float orbref_sinf(float x);  /* glibc 2.35 sinf restatement */
float orbref_cosf(float x);  /* glibc 2.35 cosf restatement */
int orbref_descriptor_distance(const uint8_t* a, const uint8_t* b);
/* one rBRIEF descriptor: img must be the blurred level, (cx, cy) integral */
void orbref_orb_descriptor(const uint8_t* blurred, size_t step, int cx, int cy,
                           float angle_deg, uint8_t* desc32);
float orbref_ic_angle(const uint8_t* img, size_t step, int cx, int cy);

/* --- matcher --------------------------------------------------------- */
/* ORBmatcher::SearchForInitialization (ORBmatcher.cpp:474-590) for a frame
 * pair with no distortion (mvKeysUn == mvKeys, image bounds [0,W]x[0,H]).
 * prev_xy: float[2*n1], updated in place (vbPrevMatched).  matches12: int[n1].
 * check_ori: rotation-consistency test; histo_bug: use the annotated tree's
 * factor 1/HISTO_LENGTH instead of HISTO_LENGTH/360.  Returns nmatches. */
int orbref_search_for_initialization(const orbref_kp* kps1, const uint8_t* desc1, int n1,
                                     const orbref_kp* kps2, const uint8_t* desc2, int n2,
                                     float min_x, float max_x, float min_y, float max_y,
                                     float* prev_xy, int window,
                                     float nnratio, int check_ori, int histo_bug,
                                     int* matches12);

/* --- RANSAC (ransac_ref.cpp) ------------------------------------------- */
/* Sim3Solver::iterate (Sim3Solver.cpp:147-221) for one solver over n_hyp
 * given triplets (samples: 3 ints per hypothesis, indices into 0..n-1).
 * X1, X2: float[3] per point; maxerr1/2: float per point; K: fx fy cx cy.
 * out_ints = {found, consumed, best_inliers, best_hyp}; T12 (4x4 row-major),
 * R12, t12, s12 and inliers (byte per point) written when best_hyp >= 0. */
int orbref_sim3_ransac(int n, const float* X1, const float* X2, const float* maxerr1, const float* maxerr2,
                       const float* K1, const float* K2, int fix_scale, int min_inliers, int best_inliers, int n_hyp,
                       const int* samples, int* out_ints, float* out_T12, float* out_R12, float* out_t12,
                       float* out_s12, uint8_t* inliers);

/* --- stereo (stereo_ref.cpp) -------------------------------------------- */
/* Frame::ComputeStereoMatches (Frame.cpp:540-748) over the keypoints and the
 * pyramids the two extractors' last orbref_extract calls left (the left and
 * right ORBextractor of a stereo Frame).  Same spec as oracle/stereo_ref.py.
 * uright / depth: float[nL]. */
void orbref_stereo_matches(const orbref_extractor* exL, const orbref_extractor* exR, const orbref_kp* kpsL,
                           const uint8_t* descL, int nL, const orbref_kp* kpsR, const uint8_t* descR, int nR,
                           float bf, float min_z, float* uright, float* depth);

/* --- loop closure (loop_ref.cpp) ------------------------------------------ */
typedef struct orbref_vocabulary orbref_vocabulary;
orbref_vocabulary* orbref_vocabulary_create(int k, int L, int n, const int32_t* parent, const int32_t* is_leaf,
                                            const uint8_t* desc, const double* weight);
void orbref_vocabulary_destroy(orbref_vocabulary* voc);
void orbref_vocabulary_transform(const orbref_vocabulary* voc, const uint8_t* desc, int n, int levelsup,
                                 int* words, int* nodes, double* weights);
int orbref_search_by_bow_kf_kf(const orbref_vocabulary* voc, const uint8_t* d1, const float* a1, const uint8_t* v1,
                               int n1, const uint8_t* d2, const float* a2, const uint8_t* v2, int n2,
                               float nnratio, int check_ori, int* match);
int orbref_compute_sim3_query(const orbref_vocabulary* voc, int n_kp, const uint8_t* desc, const float* angle,
                              const int32_t* octave, const uint8_t* valid, const float* mp_world, const float* Tcw,
                              const float* K, const float* sigma2, int cur, const int* cands, int n_cand,
                              unsigned seed, int fix_scale, int* out, int* nmatches);
int orbref_compute_sim3_query_ex(const orbref_vocabulary* voc, int n_kp, const uint8_t* desc, const float* angle,
                                 const int32_t* octave, const uint8_t* valid, const float* mp_world,
                                 const float* Tcw, const float* K, const float* sigma2, int cur, const int* cands,
                                 int n_cand, unsigned seed, int fix_scale, int* out, int* nmatches, int* m12_out,
                                 float* pose, int* cand_state, int* rand_after);

#ifdef __cplusplus
}
#endif
#endif
