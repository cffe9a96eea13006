// Initializer.h -- drop-in replacement for ORB_SLAM2::Initializer
// (reference: ORB-SLAM2/include/Initializer.h:33-98, src/Initializer.cpp)
// running on the MI355X through orbgpu_init_initialize (include/orbgpu_init.h).
// Header-only; link liborbgpu.so.
//
//   Initializer(const Frame& ReferenceFrame, float sigma = 1.0, int iterations = 200)   :41
//   bool Initialize(const Frame& CurrentFrame, const vector<int>& vMatches12,
//                   cv::Mat& R21, cv::Mat& t21, vector<cv::Point3f>& vP3D,
//                   vector<bool>& vbTriangulated)                                        :45
// Tracking::MonocularInitialization (Tracking.cpp:755-820) compiles unchanged.
// The minimal sets come from the process-wide orbgpu_rand stream after
// SeedRandOnce(0), as the reference's DUtils::Random; every hypothesis of
// FindHomography / FindFundamental is built and scored on the GPU in one
// launch each, and ReconstructH / ReconstructF's CheckRT runs there too.
// The Frame type is a template parameter of the members (mvKeysUn, mK read).
#ifndef ORBSLAM2_AMD_INITIALIZER_H
#define ORBSLAM2_AMD_INITIALIZER_H

#ifdef ORBGPU_CV_HEADER
#include ORBGPU_CV_HEADER
#else
#include <opencv2/core/core.hpp>
#endif

#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu_init.h"
#include "Device.h"

namespace ORB_SLAM2 {

class Initializer {
public:
    template <class FrameT>
    // device (adapter-only, Device.h): the GPU Initialize() runs on (-1: the thread's)
    Initializer(const FrameT& ReferenceFrame, float sigma = 1.0, int iterations = 200, int device = -1)
        : device_(device), mSigma(sigma), mSigma2(sigma * sigma), mMaxIterations(iterations) {
        const cv::Mat& K = ReferenceFrame.mK;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) mK[3 * r + c] = K.template at<float>(r, c);
        mvKeys1 = ReferenceFrame.mvKeysUn;
    }

    template <class FrameT>
    bool Initialize(const FrameT& CurrentFrame, const std::vector<int>& vMatches12, cv::Mat& R21, cv::Mat& t21,
                    std::vector<cv::Point3f>& vP3D, std::vector<bool>& vbTriangulated) {
        const std::vector<cv::KeyPoint>& k2 = CurrentFrame.mvKeysUn;
        const int n1 = (int)mvKeys1.size(), n2 = (int)k2.size();
        if ((int)vMatches12.size() != n1) throw std::invalid_argument("vMatches12 must have one entry per reference keypoint");
        // Fewer than 8 matches: the reference's 8-point draws would index an empty vector
        // (Initializer.cpp:104-115; Tracking only calls with >= 100 matches).  Return false with
        // R21 / t21 / vP3D untouched rather than throw out of the tracking thread.
        int nmatched = 0;
        for (int i = 0; i < n1; ++i) nmatched += vMatches12[i] >= 0;
        if (nmatched < 8) return false;
        std::vector<float> p1(2 * (size_t)n1), p2(2 * (size_t)n2);
        for (int i = 0; i < n1; ++i) {
            p1[2 * i] = mvKeys1[i].pt.x;
            p1[2 * i + 1] = mvKeys1[i].pt.y;
        }
        for (int i = 0; i < n2; ++i) {
            p2[2 * i] = k2[i].pt.x;
            p2[2 * i + 1] = k2[i].pt.y;
        }
        orbgpu_init_reconstruction rec;
        float rh = 0.f;
        int model = 0;
        std::vector<float> p3d(3 * (size_t)(n1 > 0 ? n1 : 1));
        std::vector<unsigned char> tri(n1 > 0 ? n1 : 1);
        const orbslam2_amd::DeviceGuard device_guard(device_);
        const int rc = orbgpu_init_initialize(p1.data(), n1, p2.data(), n2, vMatches12.data(), mK, mSigma,
                                              mMaxIterations, &rec, &rh, &model, p3d.data(), tri.data());
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
        mRH = rh;
        mModel = model;
        if (!rec.ok) return false;  // R21 / t21 / vP3D untouched, as the reference's false returns
        R21 = cv::Mat(3, 3, CV_32F);
        t21 = cv::Mat(3, 1, CV_32F);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) R21.at<float>(r, c) = rec.R21[3 * r + c];
            t21.at<float>(r) = rec.t21[r];
        }
        vP3D.resize(n1);
        vbTriangulated.assign(n1, false);
        for (int i = 0; i < n1; ++i) {
            vP3D[i] = cv::Point3f(p3d[3 * i], p3d[3 * i + 1], p3d[3 * i + 2]);
            vbTriangulated[i] = tri[i] != 0;
        }
        return true;
    }

    // Extension (not in the reference): the last call's RH and model (0 H, 1 F).
    float mRH = 0.f;
    int mModel = -1;

private:
    int device_ = -1;
    std::vector<cv::KeyPoint> mvKeys1;
    float mK[9];
    float mSigma, mSigma2;
    int mMaxIterations;
};

}  // namespace ORB_SLAM2

#endif
