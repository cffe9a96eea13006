/*
 * orbgpu_bow.h -- C ABI of the bag-of-words path: DBoW2 vocabulary,
 * TemplatedVocabulary::transform (word + direct-index node per descriptor,
 * BowVector, FeatureVector) and ORBmatcher::SearchByBoW.
 *
 * Reference (paths relative to /root/reference/ORB-SLAM2):
 *   TemplatedVocabulary::loadFromTextFile  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1359-1448
 *   TemplatedVocabulary::transform         TemplatedVocabulary.h:1151-1283
 *   BowVector::addWeight/normalize         Thirdparty/DBoW2/DBoW2/BowVector.cpp:34-90
 *   FeatureVector::addFeature              Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45
 *   Frame::ComputeBoW (levelsup 4)         src/Frame.cpp:452-460
 *   ORBmatcher::SearchByBoW(KF, F)         src/ORBmatcher.cpp:205-348
 *   ORBmatcher::SearchByBoW(KF1, KF2)      src/ORBmatcher.cpp:604-743
 *   ORBmatcher::SearchForTriangulation     src/ORBmatcher.cpp:755-951 (+ CheckDistEpipolarLine :166-190)
 *   TemplatedVocabulary::score / the scoring loops of KeyFrameDatabase::
 *   DetectLoopCandidates / DetectRelocalizationCandidates
 *                                          TemplatedVocabulary.h:1222-1227, ScoringObject.cpp:23-313,
 *                                          src/KeyFrameDatabase.cpp:96-330
 *
 * Layouts.  A FeatureVector is returned as CSR: node ids ascending
 * (fv_nodes[0..fv_n)), fv_offsets[0..fv_n] into fv_features (feature
 * indices in insertion = ascending order).  A BowVector as parallel arrays
 * of word ids ascending and double weights.
 */
#ifndef ORBGPU_BOW_H
#define ORBGPU_BOW_H

#include <stddef.h>
#include <stdint.h>

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbgpu_vocabulary orbgpu_vocabulary;

typedef struct orbgpu_vocabulary_info {
    int k, L;            /* branching factor, depth                          */
    int scoring;         /* DBoW2 ScoringType: 0 L1 .. 5 DOT_PRODUCT          */
    int weighting;       /* DBoW2 WeightingType: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY */
    int n_nodes, n_words;
} orbgpu_vocabulary_info;

/* loadFromTextFile semantics, including the reference's loop over
 * `while(!f.eof()) getline(...)`: a trailing newline adds one childless,
 * zero-descriptor, zero-weight node under the root.  ORBGPU_ERR_ARG for a
 * header outside the reference's accepted ranges. */
int orbgpu_vocabulary_load_text(const char* path, orbgpu_vocabulary** out);
/* loadFromBinaryFile semantics (TemplatedVocabulary.h:1477-1522; the format
 * saveToBinaryFile writes, :1527-1548): weights are the file's floats; the
 * reference's `while(!f.eof())` loop processes the last record twice, so the
 * last node appears twice under its parent (the copy never wins the strict
 * minimum of transform's descent) and, when it is a leaf, adds one word; the
 * node table holds nb_nodes + 1 entries.  ORBGPU_ERR_ARG for a short header,
 * k/L/scoring/weighting outside the text loader's ranges, records under 41
 * bytes, more records than nb_nodes or a parent that is not an earlier node
 * (the reference's undefined behaviour in those cases). */
int orbgpu_vocabulary_load_binary(const char* path, orbgpu_vocabulary** out);
/* From node arrays in file order: node i+1 has parent[i], is_leaf[i],
 * desc[32*i..], weight[i] (the root, node 0, is implicit). */
int orbgpu_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes_without_root,
                             const int* parent, const int* is_leaf, const uint8_t* desc, const double* weight,
                             orbgpu_vocabulary** out);
int orbgpu_vocabulary_destroy(orbgpu_vocabulary* voc);
int orbgpu_vocabulary_get_info(const orbgpu_vocabulary* voc, orbgpu_vocabulary_info* info);

/* transform(features, BowVector, FeatureVector, levelsup) for a batch of
 * frames: frame b has d_counts[b] descriptors at d_desc + b*stride*32.
 * Per feature (at + b*stride): word id, direct-index node, weight (0 for a
 * stopped word).  Per frame: FeatureVector CSR (fv_nodes/fv_features at
 * + b*stride, fv_offsets at + b*(stride+1), count d_fv_n[b]) and BowVector
 * (bow_words/bow_values at + b*stride, count d_bow_n[b]).  stride <= 4096;
 * a frame with d_counts[b] > stride is rejected (fv_n = bow_n = -1). */
int orbgpu_bow_transform_batch_device(const orbgpu_vocabulary* voc, int batch, const uint8_t* d_desc,
                                      const int* d_counts, int stride, int levelsup, int* d_word, int* d_node,
                                      double* d_weight, int* d_fv_nodes, int* d_fv_offsets, int* d_fv_features,
                                      int* d_fv_n, int* d_bow_words, double* d_bow_values, int* d_bow_n,
                                      void* stream);
/* Host form for one frame (outputs sized n, fv_offsets n+1). */
int orbgpu_bow_transform(const orbgpu_vocabulary* voc, int n, const uint8_t* desc, int levelsup, int* word,
                         int* node, double* weight, int* fv_nodes, int* fv_offsets, int* fv_features, int* fv_n,
                         int* bow_words, double* bow_values, int* bow_n);

/* ---------------------------------------------------------------------- */
/* SearchByBoW                                                              */
/* ---------------------------------------------------------------------- */
#define ORBGPU_BOW_KF_F 0   /* SearchByBoW(KF, F): A = KF, B = F            */
#define ORBGPU_BOW_KF_KF 1  /* SearchByBoW(KF1, KF2): A = KF1, B = KF2      */

/* One frame of a SearchByBoW pair.  Feature i of the frame: descriptor
 * desc + 32*i, angle[i] (KeyPoint::angle), valid[i] (the frame's MapPoint i
 * exists and is not bad; for F in KF_F mode pass all ones).  FeatureVector
 * in the CSR layout above. */
typedef struct orbgpu_bow_frame {
    int n;                          /* features                           */
    int fv_n;                       /* FeatureVector nodes                */
    const int* fv_nodes;
    const int* fv_offsets;
    const int* fv_features;
    const uint8_t* desc;
    const float* angle;
    const uint8_t* valid;
} orbgpu_bow_frame;

/* Batched, HBM-resident (frames and everything they point to on the
 * device).  Pair p: frames d_a[p], d_b[p]; output d_match + p*stride:
 *   KF_F : match[iF]  = KF feature index or -1  (vpMapPointMatches, size F.N)
 *   KF_KF: match[i1]  = KF2 feature index or -1 (vpMatches12, size KF1.N)
 * d_nmatches[p] = the return value, or -1 for a pair rejected because a
 * frame has more than `stride` features (never truncated). */
int orbgpu_search_by_bow_batch_device(int mode, int batch, const orbgpu_bow_frame* d_a, const orbgpu_bow_frame* d_b,
                                      float nnratio, int check_ori, int stride, int* d_match, int* d_nmatches,
                                      void* stream);
/* Host form for one pair (host arrays; match sized as above). */
int orbgpu_search_by_bow(int mode, const orbgpu_bow_frame* a, const orbgpu_bow_frame* b, float nnratio,
                         int check_ori, int* match, int* nmatches);

/* ---------------------------------------------------------------------- */
/* Keyframe database scoring                                               */
/* ---------------------------------------------------------------------- */
/* One query BowVector (q_words ascending, q_values) against nkf keyframes'
 * BowVectors (CSR: keyframe k's words db_words[db_offsets[k] ..
 * db_offsets[k+1]) ascending, values in db_values).  Per keyframe: the
 * number of words it shares with the query (KeyFrameDatabase's
 * mnLoopWords / mnRelocWords over the inverted file, KeyFrameDatabase.cpp:
 * 107-125, 250-262) and TemplatedVocabulary::score(query, kf) for the
 * vocabulary's scoring type (0 L1 .. 5 DOT_PRODUCT; ScoringObject.cpp
 * 23-313), summed in the reference's word order (bit-exact; KL uses the
 * device log).  The candidate selection (0.8 * max common words, minScore,
 * covisibility groups) stays with the caller. */
int orbgpu_bow_score_batch_device(int scoring, const int* d_q_words, const double* d_q_values, int nq, int nkf,
                                  const int* d_db_offsets, const int* d_db_words, const double* d_db_values,
                                  int* d_common, double* d_scores, void* stream);
/* Host form (host arrays). */
int orbgpu_bow_score(int scoring, const int* q_words, const double* q_values, int nq, int nkf,
                     const int* db_offsets, const int* db_words, const double* db_values, int* common,
                     double* scores);

/* ---------------------------------------------------------------------- */
/* SearchForTriangulation (LocalMapping::CreateNewMapPoints,               */
/* LocalMapping.cpp:355-360)                                               */
/* ---------------------------------------------------------------------- */
/* One keyframe pair.  kf1 / kf2: FeatureVector CSR, descriptors,
 * angle[i] = mvKeysUn[i].angle, valid[i] = 1 when the keyframe has NO
 * MapPoint at i (GetMapPoint(idx) == NULL: only untracked keypoints are
 * matched).  kps = mvKeysUn (x, y, octave read), u_right = mvuRight (NULL =
 * monocular, all -1).  The epipole is computed from Cw1 (pKF1's camera
 * centre) and pKF2's pose as the reference does (:763-770). */
typedef struct orbgpu_triangulation_pair {
    orbgpu_bow_frame kf1, kf2;
    const orbgpu_keypoint* kps1;
    const orbgpu_keypoint* kps2;
    const float* u_right1;
    const float* u_right2;
    float F12[9];              /* row-major, F12.at<float>(r, c) = F12[3r + c] */
    float Cw1[3];              /* pKF1->GetCameraCenter()                     */
    float T2w[12];             /* pKF2 [R2w | t2w], row-major 3 x 4           */
    float fx2, fy2, cx2, cy2;  /* pKF2 intrinsics                             */
    float scale_factors2[16];  /* pKF2->mvScaleFactors                        */
    float level_sigma2_2[16];  /* pKF2->mvLevelSigma2                         */
    int only_stereo;           /* bOnlyStereo                                 */
} orbgpu_triangulation_pair;

/* Batched (pairs and everything they point to on the device).  Pair p
 * writes d_match12 + p*stride: kf1.n ints, the KF2 keypoint matched to each
 * KF1 keypoint after the rotation cull, or -1 (vMatchedPairs = the (i, m[i])
 * with m[i] >= 0 in increasing i); d_nmatches[p] = the return value, -1 for
 * a pair rejected because a keyframe has more than `stride` features. */
int orbgpu_search_for_triangulation_batch_device(int batch, const orbgpu_triangulation_pair* d_pairs, int check_ori,
                                                 int stride, int* d_match12, int* d_nmatches, void* stream);
/* Host form for one pair (host arrays; match12 sized kf1.n). */
int orbgpu_search_for_triangulation(const orbgpu_triangulation_pair* pair, int check_ori, int* match12,
                                    int* nmatches);

#ifdef __cplusplus
}
#endif
#endif
