// StereoMatcher.h -- Frame::ComputeStereoMatches (reference:
// ORB-SLAM2/src/Frame.cpp:540-748, declared include/Frame.h:121) for the
// stereo Frame built by two drop-in ORBextractor objects (Frame.cpp:84-98),
// on the MI355X through orbgpu_stereo_matches_pair (include/orbgpu_stereo.h).
// Header-only; link liborbgpu.so.
//
// The reference's ComputeStereoMatches reads both extractors' host
// mvImagePyramid for the 11x11 SAD search; here the SAD search reads the
// levels the two extractors left in HBM, so no pyramid ever crosses PCIe.
// The reference tree swaps the body of Frame::ComputeStereoMatches for one
// call:
//
//   void Frame::ComputeStereoMatches() {
//       ORB_SLAM2::ComputeStereoMatchesGPU(mpORBextractorLeft, mpORBextractorRight, mvKeys, mDescriptors,
//                                          mvKeysRight, mDescriptorsRight, mbf, mb, mvuRight, mvDepth);
//   }
//
// Same outputs as the reference (mvuRight / mvDepth of size N, -1 where
// unmatched); the spec decisions for the cases the reference leaves
// undefined are in DESIGN.md §5c.  Failures throw std::runtime_error.
#ifndef ORBSLAM2_AMD_STEREOMATCHER_H
#define ORBSLAM2_AMD_STEREOMATCHER_H

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu_stereo.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {

namespace stereo_detail {
inline void to_raw(const std::vector<cv::KeyPoint>& in, std::vector<orbgpu_keypoint>& out) {
    out.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const cv::KeyPoint& k = in[i];
        out[i] = orbgpu_keypoint{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave, k.class_id};
    }
}
inline void to_rows(const cv::Mat& d, size_t n, std::vector<unsigned char>& out) {
    out.resize(n * 32);
    for (size_t i = 0; i < n; ++i) std::memcpy(&out[i * 32], d.ptr<unsigned char>((int)i), 32);
}
}  // namespace stereo_detail

// mb is the baseline as Frame holds it when the reference calls
// ComputeStereoMatches (0 in the stereo constructor: Frame.cpp:67, :98, :123).
inline void ComputeStereoMatchesGPU(ORBextractor* left, ORBextractor* right, const std::vector<cv::KeyPoint>& keysL,
                                    const cv::Mat& descL, const std::vector<cv::KeyPoint>& keysR,
                                    const cv::Mat& descR, float mbf, float mb, std::vector<float>& mvuRight,
                                    std::vector<float>& mvDepth) {
    const size_t N = keysL.size();
    mvuRight = std::vector<float>(N, -1.0f);  // Frame.cpp:542-543
    mvDepth = std::vector<float>(N, -1.0f);
    if (N == 0) return;
    thread_local std::vector<orbgpu_keypoint> kl, kr;
    thread_local std::vector<unsigned char> dl, dr;
    stereo_detail::to_raw(keysL, kl);
    stereo_detail::to_raw(keysR, kr);
    stereo_detail::to_rows(descL, N, dl);
    stereo_detail::to_rows(descR, keysR.size(), dr);
    if (orbgpu_stereo_matches_pair(left->handle(), right->handle(), kl.data(), dl.data(), (int)N, kr.data(),
                                   dr.data(), (int)kr.size(), mbf, mb, mvuRight.data(), mvDepth.data()) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
}

}  // namespace ORB_SLAM2

#endif
