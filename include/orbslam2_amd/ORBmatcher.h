// ORBmatcher.h -- MI355X bodies for the ORB_SLAM2::ORBmatcher member
// functions on the hot path, for a maintainer to call from the reference's
// ORBmatcher.cpp.  Header-only over include/orbgpu.h.
//
//   SearchForInitialization  ORBmatcher.h:108, ORBmatcher.cpp:474-590
//
// FrameT is ORB_SLAM2::Frame (or anything with the same members):
// mvKeysUn (std::vector<cv::KeyPoint>), mDescriptors (N x 32 CV_8U) and the
// grid bounds mnMinX, mnMaxX, mnMinY, mnMaxY (Frame.h:190-193).
#ifndef ORBSLAM2_AMD_ORBMATCHER_H
#define ORBSLAM2_AMD_ORBMATCHER_H

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

namespace orbslam2_amd {

namespace detail {
inline void check(int rc) {
    if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
}
inline void pack_keys(const std::vector<cv::KeyPoint>& in, std::vector<orbgpu_keypoint>& out) {
    out.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const cv::KeyPoint& k = in[i];
        out[i] = orbgpu_keypoint{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave, k.class_id};
    }
}
inline void pack_desc(const cv::Mat& m, size_t n, std::vector<unsigned char>& out) {
    if (n && (m.rows != (int)n || m.cols != 32)) throw std::invalid_argument("descriptors must be N x 32 CV_8U");
    out.resize(n * 32);
    for (size_t i = 0; i < n; ++i) std::memcpy(&out[i * 32], m.ptr<unsigned char>((int)i), 32);
}
}  // namespace detail

// ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, vbPrevMatched,
// vnMatches12, windowSize).  annotatedHisto selects the annotated tree's
// rotation-bin factor ("HISTO factor").
template <class FrameT>
int SearchForInitialization(float nnratio, bool checkOri, FrameT& F1, FrameT& F2,
                            std::vector<cv::Point2f>& vbPrevMatched, std::vector<int>& vnMatches12,
                            int windowSize = 10, bool annotatedHisto = false) {
    const size_t n1 = F1.mvKeysUn.size(), n2 = F2.mvKeysUn.size();
    if (vbPrevMatched.size() != n1) throw std::invalid_argument("vbPrevMatched size != F1 keypoints");
    std::vector<orbgpu_keypoint> k1, k2;
    std::vector<unsigned char> d1, d2;
    detail::pack_keys(F1.mvKeysUn, k1);
    detail::pack_keys(F2.mvKeysUn, k2);
    detail::pack_desc(F1.mDescriptors, n1, d1);
    detail::pack_desc(F2.mDescriptors, n2, d2);
    std::vector<float> prev(n1 * 2);
    for (size_t i = 0; i < n1; ++i) {
        prev[2 * i] = vbPrevMatched[i].x;
        prev[2 * i + 1] = vbPrevMatched[i].y;
    }
    vnMatches12.assign(n1, -1);
    const orbgpu_grid_bounds bd{F2.mnMinX, F2.mnMaxX, F2.mnMinY, F2.mnMaxY};
    const int flags = (checkOri ? ORBGPU_MATCH_CHECK_ORI : 0) | (annotatedHisto ? ORBGPU_MATCH_ANNOTATED_HISTO : 0);
    int nmatches = 0;
    detail::check(orbgpu_search_for_initialization(bd, k1.data(), d1.data(), (int)n1, k2.data(), d2.data(), (int)n2,
                                                   prev.data(), windowSize, nnratio, flags, vnMatches12.data(),
                                                   &nmatches));
    for (size_t i = 0; i < n1; ++i) vbPrevMatched[i] = cv::Point2f(prev[2 * i], prev[2 * i + 1]);
    return nmatches;
}

}  // namespace orbslam2_amd

#endif
