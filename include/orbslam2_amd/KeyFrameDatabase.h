// KeyFrameDatabase.h -- drop-in for ORB_SLAM2::KeyFrameDatabase (reference:
// ORB-SLAM2/include/KeyFrameDatabase.h:42-70, src/KeyFrameDatabase.cpp) whose
// BoW similarity scores run on the MI355X (orbgpu_bow_score, include/orbgpu_bow.h).
// Header-only; link liborbgpu.so.
//
// The inverted file, the shared-word counts, the 0.8 x max-common-words
// filter, the covisibility accumulation and the 0.75 x best-group cut are the
// reference's, in its order and with its KeyFrame fields (mnLoopQuery,
// mnLoopWords, mLoopScore, mnRelocQuery, mnRelocWords, mRelocScore); the
// TemplatedVocabulary::score calls of all retained keyframes are one GPU
// launch per query.  In the reference tree the replacement
// include/KeyFrameDatabase.h is
//
//     class KeyFrame; class Frame;
//     class KeyFrameDatabase : public orbslam2_amd::KeyFrameDatabaseT<KeyFrame, Frame> {
//     public:
//         KeyFrameDatabase(const ORBVocabulary& voc) : KeyFrameDatabaseT(voc) {}
//     };
//
// (the members instantiate where KeyFrame and Frame are complete, in
// Tracking.cc / LoopClosing.cc), see INTEGRATION.md section 8e.
#ifndef ORBSLAM2_AMD_KEYFRAMEDATABASE_H
#define ORBSLAM2_AMD_KEYFRAMEDATABASE_H

#include <list>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../orbgpu_bow.h"

namespace orbslam2_amd {

template <class KeyFrame, class Frame>
class KeyFrameDatabaseT {
public:
    // voc: a DBoW2 TemplatedVocabulary (size(), getScoringType())
    template <class Voc>
    explicit KeyFrameDatabaseT(const Voc& voc) : mnWords(voc.size()), mScoring((int)voc.getScoringType()) {
        mvInvertedFile.resize(mnWords);
    }

    void add(KeyFrame* pKF) {
        std::unique_lock<std::mutex> lock(mMutex);
        for (auto vit = pKF->mBowVec.begin(), vend = pKF->mBowVec.end(); vit != vend; vit++)
            mvInvertedFile[vit->first].push_back(pKF);
    }

    void erase(KeyFrame* pKF) {
        std::unique_lock<std::mutex> lock(mMutex);
        for (auto vit = pKF->mBowVec.begin(), vend = pKF->mBowVec.end(); vit != vend; vit++) {
            std::list<KeyFrame*>& lKFs = mvInvertedFile[vit->first];
            for (auto lit = lKFs.begin(), lend = lKFs.end(); lit != lend; lit++)
                if (pKF == *lit) {
                    lKFs.erase(lit);
                    break;
                }
        }
    }

    void clear() {
        mvInvertedFile.clear();
        mvInvertedFile.resize(mnWords);
    }

    // KeyFrameDatabase.cpp:96-211
    std::vector<KeyFrame*> DetectLoopCandidates(KeyFrame* pKF, float minScore) {
        const auto spConnectedKeyFrames = pKF->GetConnectedKeyFrames();
        std::list<KeyFrame*> lKFsSharingWords;
        {
            std::unique_lock<std::mutex> lock(mMutex);
            for (auto vit = pKF->mBowVec.begin(), vend = pKF->mBowVec.end(); vit != vend; vit++) {
                std::list<KeyFrame*>& lKFs = mvInvertedFile[vit->first];
                for (KeyFrame* pKFi : lKFs) {
                    if (pKFi->mnLoopQuery != pKF->mnId) {
                        pKFi->mnLoopWords = 0;
                        if (!spConnectedKeyFrames.count(pKFi)) {
                            pKFi->mnLoopQuery = pKF->mnId;
                            lKFsSharingWords.push_back(pKFi);
                        }
                    }
                    pKFi->mnLoopWords++;
                }
            }
        }
        if (lKFsSharingWords.empty()) return std::vector<KeyFrame*>();
        int maxCommonWords = 0;
        for (KeyFrame* k : lKFsSharingWords)
            if (k->mnLoopWords > maxCommonWords) maxCommonWords = k->mnLoopWords;
        const int minCommonWords = maxCommonWords * 0.8f;
        std::vector<KeyFrame*> scored;
        for (KeyFrame* k : lKFsSharingWords)
            if (k->mnLoopWords > minCommonWords) scored.push_back(k);
        const std::vector<double> sc = Scores(pKF->mBowVec, scored);
        std::list<std::pair<float, KeyFrame*> > lScoreAndMatch;
        for (size_t i = 0; i < scored.size(); ++i) {
            const float si = (float)sc[i];
            scored[i]->mLoopScore = si;
            if (si >= minScore) lScoreAndMatch.push_back(std::make_pair(si, scored[i]));
        }
        if (lScoreAndMatch.empty()) return std::vector<KeyFrame*>();
        std::list<std::pair<float, KeyFrame*> > lAccScoreAndMatch;
        float bestAccScore = minScore;
        for (auto& it : lScoreAndMatch) {
            KeyFrame* pKFi = it.second;
            const std::vector<KeyFrame*> vpNeighs = pKFi->GetBestCovisibilityKeyFrames(10);
            float bestScore = it.first, accScore = it.first;
            KeyFrame* pBestKF = pKFi;
            for (KeyFrame* pKF2 : vpNeighs)
                if (pKF2->mnLoopQuery == pKF->mnId && pKF2->mnLoopWords > minCommonWords) {
                    accScore += pKF2->mLoopScore;
                    if (pKF2->mLoopScore > bestScore) {
                        pBestKF = pKF2;
                        bestScore = pKF2->mLoopScore;
                    }
                }
            lAccScoreAndMatch.push_back(std::make_pair(accScore, pBestKF));
            if (accScore > bestAccScore) bestAccScore = accScore;
        }
        return Retain(lAccScoreAndMatch, 0.75f * bestAccScore);
    }

    // KeyFrameDatabase.cpp:224-355
    std::vector<KeyFrame*> DetectRelocalizationCandidates(Frame* F) {
        std::list<KeyFrame*> lKFsSharingWords;
        {
            std::unique_lock<std::mutex> lock(mMutex);
            for (auto vit = F->mBowVec.begin(), vend = F->mBowVec.end(); vit != vend; vit++) {
                std::list<KeyFrame*>& lKFs = mvInvertedFile[vit->first];
                for (KeyFrame* pKFi : lKFs) {
                    if (pKFi->mnRelocQuery != F->mnId) {
                        pKFi->mnRelocWords = 0;
                        pKFi->mnRelocQuery = F->mnId;
                        lKFsSharingWords.push_back(pKFi);
                    }
                    pKFi->mnRelocWords++;
                }
            }
        }
        if (lKFsSharingWords.empty()) return std::vector<KeyFrame*>();
        int maxCommonWords = 0;
        for (KeyFrame* k : lKFsSharingWords)
            if (k->mnRelocWords > maxCommonWords) maxCommonWords = k->mnRelocWords;
        const int minCommonWords = maxCommonWords * 0.8f;
        std::vector<KeyFrame*> scored;
        for (KeyFrame* k : lKFsSharingWords)
            if (k->mnRelocWords > minCommonWords) scored.push_back(k);
        const std::vector<double> sc = Scores(F->mBowVec, scored);
        std::list<std::pair<float, KeyFrame*> > lScoreAndMatch;
        for (size_t i = 0; i < scored.size(); ++i) {
            const float si = (float)sc[i];
            scored[i]->mRelocScore = si;
            lScoreAndMatch.push_back(std::make_pair(si, scored[i]));
        }
        if (lScoreAndMatch.empty()) return std::vector<KeyFrame*>();
        std::list<std::pair<float, KeyFrame*> > lAccScoreAndMatch;
        float bestAccScore = 0;
        for (auto& it : lScoreAndMatch) {
            KeyFrame* pKFi = it.second;
            const std::vector<KeyFrame*> vpNeighs = pKFi->GetBestCovisibilityKeyFrames(10);
            float bestScore = it.first, accScore = bestScore;
            KeyFrame* pBestKF = pKFi;
            for (KeyFrame* pKF2 : vpNeighs) {
                if (pKF2->mnRelocQuery != F->mnId) continue;
                accScore += pKF2->mRelocScore;  // (the reference reads it even below minCommonWords)
                if (pKF2->mRelocScore > bestScore) {
                    pBestKF = pKF2;
                    bestScore = pKF2->mRelocScore;
                }
            }
            lAccScoreAndMatch.push_back(std::make_pair(accScore, pBestKF));
            if (accScore > bestAccScore) bestAccScore = accScore;
        }
        return Retain(lAccScoreAndMatch, 0.75f * bestAccScore);
    }

protected:
    // TemplatedVocabulary::score(q, kf) for every listed keyframe, one launch
    template <class BowVec>
    std::vector<double> Scores(const BowVec& q, const std::vector<KeyFrame*>& kfs) const {
        std::vector<int> qw, off(1, 0), dw;
        std::vector<double> qv, dv;
        for (auto it = q.begin(); it != q.end(); ++it) {
            qw.push_back((int)it->first);
            qv.push_back(it->second);
        }
        for (KeyFrame* k : kfs) {
            for (auto it = k->mBowVec.begin(); it != k->mBowVec.end(); ++it) {
                dw.push_back((int)it->first);
                dv.push_back(it->second);
            }
            off.push_back((int)dw.size());
        }
        std::vector<int> common(kfs.empty() ? 1 : kfs.size());
        std::vector<double> sc(kfs.empty() ? 1 : kfs.size());
        if (kfs.empty()) return std::vector<double>();
        const int rc = orbgpu_bow_score(mScoring, qw.data(), qv.data(), (int)qw.size(), (int)kfs.size(), off.data(),
                                        dw.empty() ? nullptr : dw.data(), dv.empty() ? nullptr : dv.data(),
                                        common.data(), sc.data());
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
        sc.resize(kfs.size());
        return sc;
    }

    static std::vector<KeyFrame*> Retain(const std::list<std::pair<float, KeyFrame*> >& acc, float minScoreToRetain) {
        std::set<KeyFrame*> spAlreadyAddedKF;
        std::vector<KeyFrame*> out;
        out.reserve(acc.size());
        for (const auto& it : acc)
            if (it.first > minScoreToRetain && !spAlreadyAddedKF.count(it.second)) {
                out.push_back(it.second);
                spAlreadyAddedKF.insert(it.second);
            }
        return out;
    }

    size_t mnWords;
    int mScoring;
    std::vector<std::list<KeyFrame*> > mvInvertedFile;
    std::mutex mMutex;
};

}  // namespace orbslam2_amd

#endif
