// ORBextractor.h -- drop-in replacement for ORB_SLAM2::ORBextractor
// (reference: ORB-SLAM2/include/ORBextractor.h:47-111,
// src/ORBextractor.cpp:412-1148) running on the MI355X through the C ABI in
// include/orbgpu.h.  Header-only; link liborbgpu.so.
//
// Same class name, constructor, operator() and accessors as the reference,
// so Frame.cpp / Tracking.cpp compile unchanged against it -- the stereo
// Frame's ComputeStereoMatches included.  Differences:
//  * the GPU handle is created on the first frame (its geometry is fixed by
//    the frame size) and re-created if the size changes;
//  * the pyramid stays in HBM.  mvImagePyramid is a HostPyramid: a
//    std::vector<cv::Mat> of nlevels entries (as ORBextractor.cpp:435 sizes
//    it) whose element access copies the last frame's levels from HBM on the
//    first read after each extraction.  An unmodified stereo Frame.cpp
//    (Frame.cpp:547-676, its only reader) therefore works as it is, paying one
//    device-to-host copy of the levels per frame; the build's
//    ORB_SLAM2::ComputeStereoMatchesGPU (StereoMatcher.h)
//    reads the HBM pyramids in place and never triggers the copy.
//    SetCopyPyramid(true) (or -DORBGPU_HOST_PYRAMID=1) copies eagerly after
//    every frame instead.  Level l is a tight w_l x h_l copy (the
//    reference's is a view into a bordered buffer whose border is never read
//    outside ORBextractor.cpp);
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
#include "Device.h"

#ifndef ORBGPU_HOST_PYRAMID
#define ORBGPU_HOST_PYRAMID 0
#endif

namespace ORB_SLAM2 {

// ORBextractor::mvImagePyramid (ORBextractor.h:85): the levels of the last
// extracted frame, copied from HBM when first read.  Element access
// (operator[], at, data, begin/end) fills every level at once (one pinned
// staging copy per level, one synchronisation); size()/empty() do not.
class HostPyramid : public std::vector<cv::Mat> {
    using Base = std::vector<cv::Mat>;

public:
    cv::Mat& operator[](size_t l) { fill(); return Base::operator[](l); }
    const cv::Mat& operator[](size_t l) const { fill(); return Base::operator[](l); }
    cv::Mat& at(size_t l) { fill(); return Base::at(l); }
    const cv::Mat& at(size_t l) const { fill(); return Base::at(l); }
    cv::Mat* data() { fill(); return Base::data(); }
    const cv::Mat* data() const { fill(); return Base::data(); }
    Base::iterator begin() { fill(); return Base::begin(); }
    Base::iterator end() { fill(); return Base::end(); }
    Base::const_iterator begin() const { fill(); return Base::begin(); }
    Base::const_iterator end() const { fill(); return Base::end(); }

    // number of device-to-host level copies so far (adapter tests)
    long copies() const { return copies_; }

private:
    friend class ORBextractor;
    // a new frame is in HBM: the host levels are stale until read
    void mark(orbgpu_extractor* ex, const orbgpu_extractor_info* info) {
        ex_ = ex;
        info_ = info;
        stale_ = true;
    }
    void fill() const {
        if (!stale_) return;
        stale_ = false;  // a failed copy is not retried silently
        Base& v = const_cast<HostPyramid&>(*this);
        const int L = (int)v.size();
        std::vector<uint8_t*> dst((size_t)L);
        std::vector<size_t> step((size_t)L);
        for (int l = 0; l < L; ++l) {
            v[(size_t)l].create(info_->level_height[l], info_->level_width[l], CV_8U);
            dst[(size_t)l] = v[(size_t)l].data;
            step[(size_t)l] = v[(size_t)l].step;
        }
        if (orbgpu_extractor_copy_levels(ex_, 0, dst.data(), step.data()) != ORBGPU_OK)
            throw std::runtime_error(std::string("orbgpu: mvImagePyramid copy: ") + orbgpu_last_error());
        ++copies_;
    }
    orbgpu_extractor* ex_ = nullptr;
    const orbgpu_extractor_info* info_ = nullptr;
    mutable bool stale_ = false;
    mutable long copies_ = 0;
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    // ORBextractor.cpp:412-434 -- the scale tables are set up here exactly as
    // the reference does (double chain stored as float) so the accessors work
    // before the first frame.
    // device (adapter-only, Device.h): the GPU the extractor's handle lives on (-1: the
    // creating thread's current device when the first frame arrives)
    ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniThFAST_, int minThFAST_, int device = -1)
        : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), iniThFAST(iniThFAST_),
          minThFAST(minThFAST_), device_(device) {
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
        mvImagePyramid.resize((size_t)nlevels);  // ORBextractor.cpp:435
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
        finish_frame(n, _keypoints, _descriptors);
    }

    // adapter-only: the stereo Frame's two extractions (Frame.cpp:84-87, two
    // std::threads running ExtractORB(0) / ExtractORB(1)) from the calling
    // thread -- both frames in flight on the GPU at once, no thread spawn per
    // frame (orbgpu_extract_pair).  Results as two operator() calls.
    static void ExtractPair(ORBextractor& left, ORBextractor& right, cv::InputArray imLeft, cv::InputArray imRight,
                            std::vector<cv::KeyPoint>& keysLeft, cv::OutputArray descLeft,
                            std::vector<cv::KeyPoint>& keysRight, cv::OutputArray descRight) {
        if (imLeft.empty() || imRight.empty()) {  // ORBextractor.cpp:1056, per image
            left(imLeft, cv::Mat(), keysLeft, descLeft);
            right(imRight, cv::Mat(), keysRight, descRight);
            return;
        }
        cv::Mat L = imLeft.getMat(), R = imRight.getMat();
        if (L.type() != CV_8UC1 || R.type() != CV_8UC1) throw std::invalid_argument("ORBextractor: image must be CV_8UC1");
        if (L.cols != R.cols || L.rows != R.rows) throw std::invalid_argument("ORBextractor: stereo images differ in size");
        left.ensure_handle(L.cols, L.rows);
        right.ensure_handle(R.cols, R.rows);
        for (ORBextractor* e : {&left, &right}) {
            e->kp_buf_.resize((size_t)e->info_.max_keypoints);
            e->desc_buf_.resize((size_t)e->info_.max_keypoints * 32);
        }
        int nl = 0, nr = 0;
        check(orbgpu_extract_pair(left.ex_, L.data, L.step, left.kp_buf_.data(), left.desc_buf_.data(),
                                  left.info_.max_keypoints, &nl, right.ex_, R.data, R.step, right.kp_buf_.data(),
                                  right.desc_buf_.data(), right.info_.max_keypoints, &nr, L.cols, L.rows));
        left.finish_frame(nl, keysLeft, descLeft);
        right.finish_frame(nr, keysRight, descRight);
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
    // the device the handle lives on (-1 before the first frame)
    int device() const { return ex_ ? info_.device : device_; }

    HostPyramid mvImagePyramid;

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
    // the results of the last extraction (n keypoints in kp_buf_ / desc_buf_) into the caller's
    // vectors, as ORBextractor.cpp:1069-1116 leaves them
    void finish_frame(int n, std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors) {
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
        mvImagePyramid.mark(ex_, &info_);
        if (copy_pyramid_) mvImagePyramid.fill();
    }

    static void check(int rc) {
        if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    }
    void ensure_handle(int w, int h) {
        if (ex_ && info_.width == w && info_.height == h) return;
        if (ex_) orbgpu_extractor_destroy(ex_);
        ex_ = nullptr;
        if (device_ >= 0)
            check(orbgpu_extractor_create_on_device(device_, nfeatures, (float)scaleFactor, nlevels, iniThFAST,
                                                    minThFAST, w, h, 1, &ex_));
        else
            check(orbgpu_extractor_create(nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST, w, h, 1, &ex_));
        check(orbgpu_extractor_get_info(ex_, &info_));
    }
    int device_ = -1;
    orbgpu_extractor* ex_ = nullptr;
    orbgpu_extractor_info info_{};
    std::vector<orbgpu_keypoint> kp_buf_;
    std::vector<unsigned char> desc_buf_;
    bool copy_pyramid_ = ORBGPU_HOST_PYRAMID != 0;
};

}  // namespace ORB_SLAM2

#endif
