// PnPsolver.h -- drop-in replacement for ORB_SLAM2::PnPsolver (reference:
// ORB-SLAM2/include/PnPsolver.h:59-188, src/PnPsolver.cpp:104-1080) whose
// RANSAC hypotheses (EPnP, CheckInliers, Refine) are solved and scored on
// the MI355X through include/orbgpu_ransac.h.  Header-only; link
// liborbgpu.so.
//
// Same class name and public members as the reference, so
// Tracking::Relocalization (Tracking.cpp:1786-1822) compiles unchanged:
//   PnPsolver(const Frame& F, const vector<MapPoint*>& vpMapPointMatches)   PnPsolver.h:63
//   SetRansacParameters(probability, minInliers, maxIterations, minSet, epsilon, th2)  :66-67
//   cv::Mat find(vector<bool>& vbInliers, int& nInliers)                    :69
//   cv::Mat iterate(int nIterations, bool& bNoMore, vector<bool>& vbInliers, int& nInliers)  :71
// The constructor is a template over Frame / MapPoint (the reference's
// types deduce), the class itself is not.
//
// Random stream.  The reference draws every minimal set with
// DUtils::Random::RandomInt (glibc rand()).  iterate() draws the sets of all
// hypotheses it may run from orbgpu_random_int(), evaluates them on the GPU
// in one call, then restores the stream and re-draws exactly the sets the
// sequential loop consumed -- so the stream advances as the reference's.
// INTEGRATION.md routes DUtils::Random through the same orbgpu_rand stream.
#ifndef ORBSLAM2_AMD_PNPSOLVER_H
#define ORBSLAM2_AMD_PNPSOLVER_H

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

class PnPsolver {
public:
    template <class FrameT, class MapPointT>
    // device (adapter-only, Device.h): the GPU iterate() runs on (-1: the thread's)
    PnPsolver(const FrameT& F, const std::vector<MapPointT*>& vpMapPointMatches, int device = -1)
        : device_(device), mnMatches((int)vpMapPointMatches.size()) {
        // PnPsolver.cpp:104-139: correspondences of the good MapPoints
        for (size_t i = 0; i < vpMapPointMatches.size(); ++i) {
            MapPointT* pMP = vpMapPointMatches[i];
            if (!pMP || pMP->isBad()) continue;
            const cv::KeyPoint& kp = F.mvKeysUn[i];
            mvP2D.push_back(kp.pt.x);
            mvP2D.push_back(kp.pt.y);
            mvSigma2.push_back(F.mvLevelSigma2[kp.octave]);
            const cv::Mat Pos = pMP->GetWorldPos();
            for (int k = 0; k < 3; ++k) mvP3Dw.push_back(Pos.template at<float>(k));
            mvKeyPointIndices.push_back((int)i);
        }
        N = (int)mvSigma2.size();
        fu = F.fx;
        fv = F.fy;
        uc = F.cx;
        vc = F.cy;
        mvbBestInliers.assign(N, 0);
        SetRansacParameters();
    }

    // PnPsolver.cpp:159-195
    void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300, int minSet = 4,
                             float epsilon = 0.4, float th2 = 5.991) {
        mRansacProb = probability;
        mRansacMaxIts = maxIterations;
        mRansacEpsilon = epsilon;
        mRansacMinSet = minSet;
        int nMinInliers = (int)((float)N * mRansacEpsilon);
        if (nMinInliers < minInliers) nMinInliers = minInliers;
        if (nMinInliers < minSet) nMinInliers = minSet;
        mRansacMinInliers = nMinInliers;
        if (N > 0 && mRansacEpsilon < (float)mRansacMinInliers / (float)N) mRansacEpsilon = (float)mRansacMinInliers / N;
        int nIterations;
        if (mRansacMinInliers == N) {
            nIterations = 1;
        } else {
            const double v = std::ceil(std::log(1 - mRansacProb) / std::log(1 - std::pow((double)mRansacEpsilon, 3.0)));
            nIterations = (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (int)0x80000000;  // x86 cvttsd2si
        }
        mRansacMaxIts = std::max(1, std::min(nIterations, mRansacMaxIts));
        mvMaxError.resize(mvSigma2.size());
        for (size_t i = 0; i < mvSigma2.size(); ++i) mvMaxError[i] = mvSigma2[i] * th2;
    }

    cv::Mat find(std::vector<bool>& vbInliers, int& nInliers) {
        bool bFlag;
        return iterate(mRansacMaxIts, bFlag, vbInliers, nInliers);
    }

    // PnPsolver.cpp:203-301
    cv::Mat iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers) {
        bNoMore = false;
        vbInliers.clear();
        nInliers = 0;
        if (N < mRansacMinInliers) {
            bNoMore = true;
            return cv::Mat();
        }
        // while (mnIterations < mRansacMaxIts || nCurrentIterations < nIterations)
        const int n_hyp = std::max(mRansacMaxIts - mnIterations, nIterations);
        orbgpu_rand_state snap;
        orbgpu_rand_get_state(&snap);
        std::vector<int> samples;
        draw(n_hyp, samples);
        orbgpu_pnp_problem p;
        p.n = N;
        p.offset = 0;
        p.min_inliers = mRansacMinInliers;
        p.best_inliers = mnBestInliers;
        p.n_hyp = n_hyp;
        p.sample_offset = 0;
        p.fu = fu;
        p.fv = fv;
        p.uc = uc;
        p.vc = vc;
        std::vector<uint8_t> best = mvbBestInliers, refined(N > 0 ? N : 1, 0);
        if (best.empty()) best.assign(1, 0);
        orbgpu_pnp_result r;
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_pnp_ransac_batch(1, &p, N, mvP3Dw.data(), mvP2D.data(), mvMaxError.data(), n_hyp,
                                      samples.empty() ? nullptr : samples.data(), &r, best.data(), refined.data()));
        orbgpu_rand_set_state(&snap);  // consume exactly the iterations the reference ran
        draw(r.consumed, samples);
        mnIterations += r.consumed;
        mnBestInliers = r.best_inliers;
        if (r.best_hyp >= 0) {
            mvbBestInliers.assign(best.begin(), best.begin() + N);
            mBestTcw = to_mat(r.best_Tcw);
        }
        if (r.found) {
            nInliers = r.refined_inliers;
            vbInliers.assign(mnMatches, false);
            for (int i = 0; i < N; ++i)
                if (refined[i]) vbInliers[mvKeyPointIndices[i]] = true;
            return to_mat(r.refined_Tcw);
        }
        if (mnIterations >= mRansacMaxIts) {
            bNoMore = true;
            if (mnBestInliers >= mRansacMinInliers) {
                nInliers = mnBestInliers;
                vbInliers.assign(mnMatches, false);
                for (int i = 0; i < N; ++i)
                    if (mvbBestInliers[i]) vbInliers[mvKeyPointIndices[i]] = true;
                return mBestTcw.clone();
            }
        }
        return cv::Mat();
    }

    // state, exposed read-only for tests and diagnostics (not in the reference)
    int Iterations() const { return mnIterations; }
    int BestInliers() const { return mnBestInliers; }
    int MinInliers() const { return mRansacMinInliers; }
    int MaxIterations() const { return mRansacMaxIts; }
    int Correspondences() const { return N; }

private:
    int device_ = -1;
    static void check(int rc) {
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    }
    // mRansacMinSet x (RandomInt(0, size-1), swap with back, pop) per iteration (:229-244)
    void draw(int n_iter, std::vector<int>& out) const {
        out.assign((size_t)n_iter * mRansacMinSet, 0);
        std::vector<int> avail;
        for (int it = 0; it < n_iter; ++it) {
            avail.resize(N);
            for (int i = 0; i < N; ++i) avail[i] = i;
            for (int j = 0; j < mRansacMinSet; ++j) {
                const int r = orbgpu_random_int(0, (int)avail.size() - 1);
                out[(size_t)it * mRansacMinSet + j] = avail[r];
                avail[r] = avail.back();
                avail.pop_back();
            }
        }
    }
    static cv::Mat to_mat(const float T[16]) {
        cv::Mat m = cv::Mat::eye(4, 4, CV_32F);
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) m.at<float>(r, c) = T[4 * r + c];
        return m;
    }

    int mnMatches;                    // vpMapPointMatches.size()
    std::vector<float> mvP2D, mvP3Dw, mvSigma2, mvMaxError;
    std::vector<int> mvKeyPointIndices;
    std::vector<uint8_t> mvbBestInliers;
    int N = 0;
    float fu = 0, fv = 0, uc = 0, vc = 0;
    double mRansacProb = 0.99;
    int mRansacMinInliers = 8, mRansacMaxIts = 300, mRansacMinSet = 4;
    float mRansacEpsilon = 0.4f;
    int mnIterations = 0, mnBestInliers = 0;
    cv::Mat mBestTcw;
};

}  // namespace ORB_SLAM2

#endif
