// Sim3Solver.h -- drop-in replacement for ORB_SLAM2::Sim3Solver (reference:
// ORB-SLAM2/include/Sim3Solver.h:35-125, src/Sim3Solver.cpp:37-447) whose
// RANSAC hypotheses (ComputeSim3 + CheckInliers) are solved and scored on the
// MI355X through include/orbgpu_ransac.h.  Header-only; link liborbgpu.so.
//
// Same class name and public members as the reference, so
// LoopClosing::ComputeSim3 (LoopClosing.cpp:311-356) compiles unchanged:
//   Sim3Solver(KeyFrame* pKF1, KeyFrame* pKF2, const vector<MapPoint*>& vpMatched12, bool bFixScale = true)  :39
//   SetRansacParameters(probability = 0.99, minInliers = 6, maxIterations = 300)  :41
//   cv::Mat find(vector<bool>& vbInliers12, int& nInliers)                        :43
//   cv::Mat iterate(int nIterations, bool& bNoMore, vector<bool>& vbInliers, int& nInliers)  :45
//   GetEstimatedRotation / GetEstimatedTranslation / GetEstimatedScale            :47-49
// The constructor is a template over KeyFrame / MapPoint.  It reads
// GetMapPointMatches(), GetRotation(), GetTranslation(), mvKeysUn,
// mvLevelSigma2 and mK of the keyframes and GetWorldPos(), isBad(),
// GetIndexInKeyFrame() of the MapPoints, as Sim3Solver.cpp:37-107 does.
//
// Random stream: as PnPsolver.h -- speculative draws from orbgpu_random_int
// with the state restored and exactly the consumed sets re-drawn.
// For a whole ComputeSim3 (all candidates, round-robin) in one launch see
// include/orbgpu_loop.h.
#ifndef ORBSLAM2_AMD_SIM3SOLVER_H
#define ORBSLAM2_AMD_SIM3SOLVER_H

#ifdef ORBGPU_CV_HEADER
#include ORBGPU_CV_HEADER
#else
#include <opencv2/core/core.hpp>
#endif

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu_ransac.h"
#include "Device.h"

namespace ORB_SLAM2 {

class Sim3Solver {
public:
    template <class KeyFrameT, class MapPointT>
    // device (adapter-only, Device.h): the GPU iterate() runs on (-1: the thread's)
    Sim3Solver(KeyFrameT* pKF1, KeyFrameT* pKF2, const std::vector<MapPointT*>& vpMatched12,
               const bool bFixScale = true, int device = -1)
        : device_(device), mN1((int)vpMatched12.size()), mbFixScale(bFixScale) {
        const std::vector<MapPointT*> vpKeyFrameMP1 = pKF1->GetMapPointMatches();
        const cv::Mat Rcw1 = pKF1->GetRotation(), tcw1 = pKF1->GetTranslation();
        const cv::Mat Rcw2 = pKF2->GetRotation(), tcw2 = pKF2->GetTranslation();
        for (int i1 = 0; i1 < mN1; ++i1) {  // Sim3Solver.cpp:54-99
            MapPointT* pMP2 = vpMatched12[i1];
            if (!pMP2) continue;
            MapPointT* pMP1 = vpKeyFrameMP1[i1];
            if (!pMP1) continue;
            if (pMP1->isBad() || pMP2->isBad()) continue;
            const int indexKF1 = pMP1->GetIndexInKeyFrame(pKF1);
            const int indexKF2 = pMP2->GetIndexInKeyFrame(pKF2);
            if (indexKF1 < 0 || indexKF2 < 0) continue;
            const float sigmaSquare1 = pKF1->mvLevelSigma2[pKF1->mvKeysUn[indexKF1].octave];
            const float sigmaSquare2 = pKF2->mvLevelSigma2[pKF2->mvKeysUn[indexKF2].octave];
            // vector<size_t> mvnMaxError: 9.210*sigma^2 truncated (:92-93)
            mvnMaxError1.push_back((float)(size_t)(9.210 * sigmaSquare1));
            mvnMaxError2.push_back((float)(size_t)(9.210 * sigmaSquare2));
            mvnIndices1.push_back(i1);
            cam(Rcw1, tcw1, pMP1->GetWorldPos(), mvX3Dc1);  // Rcw1*X3D1w + tcw1
            cam(Rcw2, tcw2, pMP2->GetWorldPos(), mvX3Dc2);
        }
        N = (int)mvnIndices1.size();
        const cv::Mat& K1 = pKF1->mK;
        const cv::Mat& K2 = pKF2->mK;
        mK1[0] = K1.template at<float>(0, 0);
        mK1[1] = K1.template at<float>(1, 1);
        mK1[2] = K1.template at<float>(0, 2);
        mK1[3] = K1.template at<float>(1, 2);
        mK2[0] = K2.template at<float>(0, 0);
        mK2[1] = K2.template at<float>(1, 1);
        mK2[2] = K2.template at<float>(0, 2);
        mK2[3] = K2.template at<float>(1, 2);
        mvbBestInliers.assign(N > 0 ? N : 1, 0);
        SetRansacParameters();
    }

    // Sim3Solver.cpp:111-141
    void SetRansacParameters(double probability = 0.99, int minInliers = 6, int maxIterations = 300) {
        mRansacProb = probability;
        mRansacMinInliers = minInliers;
        mRansacMaxIts = maxIterations;
        int nIterations;
        if (mRansacMinInliers == N) {
            nIterations = 1;
        } else {
            const float epsilon = (float)mRansacMinInliers / (float)N;
            const double v = std::ceil(std::log(1 - mRansacProb) / std::log(1 - std::pow((double)epsilon, 3.0)));
            nIterations = (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (int)0x80000000;  // x86 cvttsd2si
        }
        mRansacMaxIts = std::max(1, std::min(nIterations, mRansacMaxIts));
        mnIterations = 0;
    }

    cv::Mat find(std::vector<bool>& vbInliers12, int& nInliers) {
        bool bFlag;
        return iterate(mRansacMaxIts, bFlag, vbInliers12, nInliers);
    }

    // Sim3Solver.cpp:147-221
    cv::Mat iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers) {
        bNoMore = false;
        vbInliers.assign(mN1, false);
        nInliers = 0;
        if (N < mRansacMinInliers) {
            bNoMore = true;
            return cv::Mat();
        }
        const int n_hyp = std::max(0, std::min(nIterations, mRansacMaxIts - mnIterations));
        orbgpu_rand_state snap;
        orbgpu_rand_get_state(&snap);
        std::vector<int> samples;
        draw(n_hyp, samples);
        orbgpu_sim3_problem p;
        p.n = N;
        p.offset = 0;
        p.fix_scale = mbFixScale ? 1 : 0;
        p.min_inliers = mRansacMinInliers;
        p.best_inliers = mnBestInliers;
        p.n_hyp = n_hyp;
        p.sample_offset = 0;
        p.pad = 0;
        for (int k = 0; k < 4; ++k) {
            p.K1[k] = mK1[k];
            p.K2[k] = mK2[k];
        }
        std::vector<uint8_t> mask = mvbBestInliers;
        orbgpu_sim3_result r;
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_sim3_ransac_batch(1, &p, N, mvX3Dc1.data(), mvX3Dc2.data(), mvnMaxError1.data(),
                                       mvnMaxError2.data(), n_hyp, samples.empty() ? nullptr : samples.data(), &r,
                                       mask.data()));
        orbgpu_rand_set_state(&snap);  // consume exactly the iterations the reference ran
        draw(r.consumed, samples);
        mnIterations += r.consumed;
        mnBestInliers = r.best_inliers;
        if (r.best_hyp >= 0) {
            mvbBestInliers = mask;
            mBestT12 = cv::Mat::eye(4, 4, CV_32F);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) mBestT12.at<float>(i, j) = r.T12[4 * i + j];
            mBestRotation = cv::Mat(3, 3, CV_32F);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) mBestRotation.at<float>(i, j) = r.R12[3 * i + j];
            mBestTranslation = cv::Mat(3, 1, CV_32F);
            for (int i = 0; i < 3; ++i) mBestTranslation.at<float>(i, 0) = r.t12[i];
            mBestScale = r.s12;
        }
        if (r.found) {
            nInliers = r.best_inliers;
            for (int i = 0; i < N; ++i)
                if (mvbBestInliers[i]) vbInliers[mvnIndices1[i]] = true;
            return mBestT12;
        }
        if (mnIterations >= mRansacMaxIts) bNoMore = true;
        return cv::Mat();
    }

    cv::Mat GetEstimatedRotation() { return mBestRotation.clone(); }
    cv::Mat GetEstimatedTranslation() { return mBestTranslation.clone(); }
    float GetEstimatedScale() { return mBestScale; }

    // state, exposed read-only for tests and diagnostics (not in the reference)
    int Iterations() const { return mnIterations; }
    int BestInliers() const { return mnBestInliers; }
    int MaxIterations() const { return mRansacMaxIts; }
    int Correspondences() const { return N; }

private:
    int device_ = -1;
    static void check(int rc) {
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    }
    // float 3x3 * 3x1 with double accumulation (OpenCV's small float gemm) + t
    static void cam(const cv::Mat& R, const cv::Mat& t, const cv::Mat& X, std::vector<float>& out) {
        for (int i = 0; i < 3; ++i) {
            const double s = (double)R.template at<float>(i, 0) * (double)X.template at<float>(0) +
                             (double)R.template at<float>(i, 1) * (double)X.template at<float>(1) +
                             (double)R.template at<float>(i, 2) * (double)X.template at<float>(2);
            out.push_back((float)s + t.template at<float>(i));
        }
    }
    // 3 x (RandomInt(0, size-1), swap with back, pop) per iteration (:172-183)
    void draw(int n_iter, std::vector<int>& out) const {
        out.assign((size_t)n_iter * 3, 0);
        std::vector<int> avail;
        for (int it = 0; it < n_iter; ++it) {
            avail.resize(N);
            for (int i = 0; i < N; ++i) avail[i] = i;
            for (int j = 0; j < 3; ++j) {
                const int r = orbgpu_random_int(0, (int)avail.size() - 1);
                out[(size_t)it * 3 + j] = avail[r];
                avail[r] = avail.back();
                avail.pop_back();
            }
        }
    }

    int mN1;
    bool mbFixScale;
    std::vector<float> mvX3Dc1, mvX3Dc2, mvnMaxError1, mvnMaxError2;
    std::vector<int> mvnIndices1;
    std::vector<uint8_t> mvbBestInliers;
    float mK1[4] = {0, 0, 0, 0}, mK2[4] = {0, 0, 0, 0};
    int N = 0;
    double mRansacProb = 0.99;
    int mRansacMinInliers = 6, mRansacMaxIts = 300;
    int mnIterations = 0, mnBestInliers = 0;
    cv::Mat mBestT12, mBestRotation, mBestTranslation;
    float mBestScale = 0.f;
};

}  // namespace ORB_SLAM2

#endif
