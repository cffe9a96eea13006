// ORBextractor.h -- drop-in replacement for ORB_SLAM2::ORBextractor
// (reference: ORB-SLAM2/include/ORBextractor.h:47-111,
// src/ORBextractor.cpp:412-1148) running on the MI355X through the C ABI in
// include/orbgpu.h.  Header-only; link liborbgpu.so.
//
// Same class name, constructor, operator() and accessors as the reference,
// so Frame.cpp / Tracking.cpp compile unchanged against it.  Differences:
//  * the GPU handle is created on the first frame (its geometry is fixed by
//    the frame size) and re-created if the size changes;
//  * the pyramid stays in HBM: mvImagePyramid is filled only when the host
//    copy is asked for (SetCopyPyramid(true), or -DORBGPU_HOST_PYRAMID=1 to
//    make that the default).  Its only reader in the reference is the stereo
//    Frame's ComputeStereoMatches (Frame.cpp:547-676), which the build
//    replaces with ORB_SLAM2::ComputeStereoMatchesGPU (StereoMatcher.h) on
//    the two extractors' HBM pyramids; a copy is then
//    8 blocking device-to-host level copies per frame for nothing.  When
//    copied, level l is a tight w_l x h_l copy (the reference's is a view
//    into a bordered buffer whose border is never read outside
//    ORBextractor.cpp);
//  * failures throw std::runtime_error carrying orbgpu_last_error() (the
//    reference asserts).
//
// OpenCV types come from <opencv2/core/core.hpp>, or from the header named
// by ORBGPU_CV_HEADER (the adapter tests use a small stand-in there).
#ifndef ORBSLAM2_AMD_ORBEXTRACTOR_H
#define ORBSLAM2_AMD_ORBEXTRACTOR_H

#ifdef ORBGPU_CV_HEADER
#include ORBGPU_CV_HEADER
#else
#include <opencv2/core/core.hpp>
#endif

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu.h"

#ifndef ORBGPU_HOST_PYRAMID
#define ORBGPU_HOST_PYRAMID 0
#endif

namespace ORB_SLAM2 {

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    // ORBextractor.cpp:412-434 -- the scale tables are set up here exactly as
    // the reference does (double chain stored as float) so the accessors work
    // before the first frame.
    ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniThFAST_, int minThFAST_)
        : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), iniThFAST(iniThFAST_),
          minThFAST(minThFAST_) {
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
    }
    ~ORBextractor() {
        if (ex_) orbgpu_extractor_destroy(ex_);
    }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // ORBextractor.cpp:1053-1117.  `mask` is ignored, as in the reference.
    void operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                    cv::OutputArray _descriptors) {
        (void)_mask;
        if (_image.empty()) return;
        cv::Mat image = _image.getMat();
        if (image.type() != CV_8UC1) throw std::invalid_argument("ORBextractor: image must be CV_8UC1");
        ensure_handle(image.cols, image.rows);
        kp_buf_.resize((size_t)info_.max_keypoints);
        desc_buf_.resize((size_t)info_.max_keypoints * 32);
        int n = 0;
        check(orbgpu_extract(ex_, image.data, image.cols, image.rows, image.step, kp_buf_.data(), desc_buf_.data(),
                             info_.max_keypoints, &n));
        _keypoints.clear();
        _keypoints.reserve((size_t)n);
        for (int i = 0; i < n; ++i) {
            const orbgpu_keypoint& k = kp_buf_[(size_t)i];
            _keypoints.push_back(cv::KeyPoint(k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id));
        }
        if (n == 0) {
            _descriptors.release();
        } else {
            _descriptors.create(n, 32, CV_8U);
            cv::Mat d = _descriptors.getMat();
            for (int i = 0; i < n; ++i) std::memcpy(d.ptr<unsigned char>(i), &desc_buf_[(size_t)i * 32], 32);
        }
        if (copy_pyramid_) {
            mvImagePyramid.resize((size_t)nlevels);
            std::vector<uint8_t*> dst((size_t)nlevels);
            std::vector<size_t> step((size_t)nlevels);
            for (int l = 0; l < nlevels; ++l) {
                mvImagePyramid[l].create(info_.level_height[l], info_.level_width[l], CV_8U);
                dst[l] = mvImagePyramid[l].data;
                step[l] = mvImagePyramid[l].step;
            }
            check(orbgpu_extractor_copy_levels(ex_, 0, dst.data(), step.data()));
        }
    }

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    // adapter-only
    void SetCopyPyramid(bool on) { copy_pyramid_ = on; }
    orbgpu_extractor* handle() { return ex_; }  // the last frame's pyramid lives here (HBM)

    std::vector<cv::Mat> mvImagePyramid;

protected:
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

private:
    static void check(int rc) {
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    }
    void ensure_handle(int w, int h) {
        if (ex_ && info_.width == w && info_.height == h) return;
        if (ex_) orbgpu_extractor_destroy(ex_);
        ex_ = nullptr;
        check(orbgpu_extractor_create(nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST, w, h, 1, &ex_));
        check(orbgpu_extractor_get_info(ex_, &info_));
    }
    orbgpu_extractor* ex_ = nullptr;
    orbgpu_extractor_info info_{};
    std::vector<orbgpu_keypoint> kp_buf_;
    std::vector<unsigned char> desc_buf_;
    bool copy_pyramid_ = ORBGPU_HOST_PYRAMID != 0;
};

}  // namespace ORB_SLAM2

#endif
