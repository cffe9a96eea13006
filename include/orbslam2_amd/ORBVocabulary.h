// ORBVocabulary.h -- drop-in for ORB_SLAM2::ORBVocabulary (reference:
// ORB-SLAM2/include/ORBVocabulary.h:29-31, the typedef of
// DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>,
// Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) whose tree lives in HBM and
// whose transform / score run on the MI355X (include/orbgpu_bow.h).
// Header-only; link liborbgpu.so.
//
// The members ORB-SLAM2 calls:
//   bool loadFromTextFile(const std::string&)          TemplatedVocabulary.h:1362   (System.cc)
//   bool loadFromBinaryFile(const std::string&)        :1478 (the binary form of the same tree)
//   void transform(features, BowVector&, FeatureVector&, levelsup) const   :1151 (Frame/KeyFrame::ComputeBoW)
//   double score(const BowVector&, const BowVector&) const                 :1222 (LoopClosing, KeyFrameDatabase)
//   unsigned size() const, ScoringType getScoringType() const              (KeyFrameDatabase)
// BowVector / FeatureVector are DBoW2's std::map types (or anything with
// clear(), operator[] and ordered iteration); features are the rows of the
// descriptor matrix as a vector of 1 x 32 CV_8U Mats (Converter::toDescriptorVector).
#ifndef ORBSLAM2_AMD_ORBVOCABULARY_H
#define ORBSLAM2_AMD_ORBVOCABULARY_H

#ifdef ORBGPU_CV_HEADER
#include ORBGPU_CV_HEADER
#else
#include <opencv2/core/core.hpp>
#endif

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu_bow.h"

namespace orbslam2_amd {

class ORBVocabulary {
public:
    ORBVocabulary() = default;
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;
    ~ORBVocabulary() {
        if (mVoc) orbgpu_vocabulary_destroy(mVoc);
    }

    // TemplatedVocabulary::loadFromTextFile: false when the file cannot be read
    // or its header is out of the reference's accepted ranges
    bool loadFromTextFile(const std::string& filename) {
        orbgpu_vocabulary* v = nullptr;
        if (orbgpu_vocabulary_load_text(filename.c_str(), &v) != ORBGPU_OK) return false;
        if (mVoc) orbgpu_vocabulary_destroy(mVoc);
        mVoc = v;
        return orbgpu_vocabulary_get_info(mVoc, &mInfo) == ORBGPU_OK;
    }

    // TemplatedVocabulary::loadFromBinaryFile (TemplatedVocabulary.h:1478); the
    // reference returns true for any file it opens, this false when the file
    // cannot be read or is malformed (include/orbgpu_bow.h)
    bool loadFromBinaryFile(const std::string& filename) {
        orbgpu_vocabulary* v = nullptr;
        if (orbgpu_vocabulary_load_binary(filename.c_str(), &v) != ORBGPU_OK) return false;
        if (mVoc) orbgpu_vocabulary_destroy(mVoc);
        mVoc = v;
        return orbgpu_vocabulary_get_info(mVoc, &mInfo) == ORBGPU_OK;
    }

    // TemplatedVocabulary::transform(features, v, fv, levelsup)
    template <class BowVector, class FeatureVector>
    void transform(const std::vector<cv::Mat>& features, BowVector& v, FeatureVector& fv, int levelsup) const {
        v.clear();
        fv.clear();
        if (!mVoc || features.empty()) return;
        const int n = (int)features.size();
        std::vector<unsigned char> desc(32 * (size_t)n);
        for (int i = 0; i < n; ++i) std::memcpy(&desc[32 * (size_t)i], features[i].template ptr<unsigned char>(0), 32);
        std::vector<int> word(n), node(n), fvn(n), fvo(n + 1), fvf(n), bw(n);
        std::vector<double> weight(n), bv(n);
        int nf = 0, nb = 0;
        check(orbgpu_bow_transform(mVoc, n, desc.data(), levelsup, word.data(), node.data(), weight.data(), fvn.data(),
                                   fvo.data(), fvf.data(), &nf, bw.data(), bv.data(), &nb));
        for (int i = 0; i < nb; ++i) v[bw[i]] = bv[i];
        for (int j = 0; j < nf; ++j) {
            auto& lst = fv[fvn[j]];
            for (int q = fvo[j]; q < fvo[j + 1]; ++q) lst.push_back((unsigned int)fvf[q]);
        }
    }

    // TemplatedVocabulary::score(a, b)
    template <class BowVector>
    double score(const BowVector& a, const BowVector& b) const {
        std::vector<int> qw, dw, off(2, 0);
        std::vector<double> qv, dv;
        for (auto it = a.begin(); it != a.end(); ++it) {
            qw.push_back((int)it->first);
            qv.push_back(it->second);
        }
        for (auto it = b.begin(); it != b.end(); ++it) {
            dw.push_back((int)it->first);
            dv.push_back(it->second);
        }
        off[1] = (int)dw.size();
        int common = 0;
        double s = 0.0;
        check(orbgpu_bow_score(mInfo.scoring, qw.empty() ? nullptr : qw.data(), qv.empty() ? nullptr : qv.data(),
                               (int)qw.size(), 1, off.data(), dw.empty() ? nullptr : dw.data(),
                               dv.empty() ? nullptr : dv.data(), &common, &s));
        return s;
    }

    unsigned int size() const { return (unsigned int)mInfo.n_words; }
    int getScoringType() const { return mInfo.scoring; }
    int getWeightingType() const { return mInfo.weighting; }
    int getBranchingFactor() const { return mInfo.k; }
    int getDepthLevels() const { return mInfo.L; }
    // the device-resident vocabulary, for the batched C ABI calls
    const orbgpu_vocabulary* handle() const { return mVoc; }

private:
    static void check(int rc) {
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    }
    orbgpu_vocabulary* mVoc = nullptr;
    orbgpu_vocabulary_info mInfo{};
};

}  // namespace orbslam2_amd

#endif
