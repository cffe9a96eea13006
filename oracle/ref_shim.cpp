/*
 * ref_shim.cpp -- C entry points into the parts of the reference that compile
 * here UNMODIFIED (TEST INFRASTRUCTURE ONLY; built by oracle/ref.mk into
 * oracle/_ref/libdbow2ref.so from the sources where they lie under
 * /root/reference; nothing of the reference is copied into this repo).
 *
 * Compiled reference files (ORB-SLAM2/Thirdparty/DBoW2/):
 *   DUtils/Random.cpp     -- DUtils::Random::SeedRand/SeedRandOnce/RandomInt (glibc rand())
 *   DUtils/Timestamp.cpp  -- needed by Random.cpp's time-seeded SeedRand()
 *   DBoW2/BowVector.cpp   -- BowVector::addWeight / addIfNotExist / normalize
 *   DBoW2/FeatureVector.cpp -- FeatureVector::addFeature
 * Not compilable here (need OpenCV): TemplatedVocabulary.h, ScoringObject.cpp,
 * FORB.cpp.  So the outer loop of TemplatedVocabulary::transform(features,
 * BowVector, FeatureVector, levelsup) (TemplatedVocabulary.h:1151-1235) and
 * the mustNormalize table of ScoringObject.h:76-91 are restated below in a
 * few lines; every BowVector / FeatureVector operation is the reference's
 * compiled code.  The per-feature (word, node, weight) come from the caller
 * (the GPU library's transform in tests/test_refpin.py).
 */
#include <cstdint>
#include <cstring>

#include "DBoW2/BowVector.h"
#include "DBoW2/FeatureVector.h"
#include "DUtils/Random.h"

extern "C" {

void ref_seed_rand_once(int seed) { DUtils::Random::SeedRandOnce(seed); }
void ref_seed_rand(int seed) { DUtils::Random::SeedRand(seed); }
int ref_random_int(int min, int max) { return DUtils::Random::RandomInt(min, max); }

/* BowVector + FeatureVector of one frame as TemplatedVocabulary::transform
 * builds them (T:1151-1235).  weighting: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY;
 * scoring: 0 L1, 1 L2, 2 CHI_SQUARE, 3 KL, 4 BHATTACHARYYA, 5 DOT_PRODUCT
 * (BowVector.h:38-55).  Outputs in map order: bow_n (word, value) pairs and
 * the FeatureVector as CSR (fv_n nodes, offsets[fv_n + 1], features). */
void ref_bow_vectors(int n, const int* words, const int* nodes, const double* weights, int weighting, int scoring,
                     int* bow_words, double* bow_values, int* bow_n, int* fv_nodes, int* fv_offsets,
                     int* fv_features, int* fv_n) {
    DBoW2::BowVector v;
    DBoW2::FeatureVector fv;
    // ScoringObject.h:76-91: every scoring normalizes (L2 for L2Scoring, L1 otherwise)
    // except DotProductScoring
    const bool must = scoring != 5;
    const DBoW2::LNorm norm = scoring == 1 ? DBoW2::L2 : DBoW2::L1;
    if (weighting == 0 || weighting == 1) {
        for (int i = 0; i < n; ++i)
            if (weights[i] > 0) {
                v.addWeight((DBoW2::WordId)words[i], weights[i]);
                fv.addFeature((DBoW2::NodeId)nodes[i], (unsigned int)i);
            }
        if (!v.empty() && !must) {
            const double nd = v.size();
            for (DBoW2::BowVector::iterator it = v.begin(); it != v.end(); it++) it->second /= nd;
        }
    } else {
        for (int i = 0; i < n; ++i)
            if (weights[i] > 0) {
                v.addIfNotExist((DBoW2::WordId)words[i], weights[i]);
                fv.addFeature((DBoW2::NodeId)nodes[i], (unsigned int)i);
            }
    }
    if (must) v.normalize(norm);
    int k = 0;
    for (const auto& e : v) {
        bow_words[k] = (int)e.first;
        bow_values[k] = e.second;
        ++k;
    }
    *bow_n = k;
    int j = 0, f = 0;
    fv_offsets[0] = 0;
    for (const auto& e : fv) {
        fv_nodes[j] = (int)e.first;
        for (unsigned int q : e.second) fv_features[f++] = (int)q;
        fv_offsets[++j] = f;
    }
    *fv_n = j;
}

}  // extern "C"
