// ORBmatcher.h -- drop-in replacement for ORB_SLAM2::ORBmatcher's hot-path
// members (reference: ORB-SLAM2/include/ORBmatcher.h:37-108,
// src/ORBmatcher.cpp) running on the MI355X through the C ABI in
// include/orbgpu.h, orbgpu_bow.h and orbgpu_proj.h.  Header-only; link
// liborbgpu.so.
//
// Same class name, constructor, constants and member signatures as the
// reference, so Tracking.cpp / LoopClosing.cpp / LocalMapping.cpp calls
// compile unchanged:
//   ORBmatcher(float nnratio = 0.6, bool checkOri = true)         ORBmatcher.h:41
//   static int DescriptorDistance(const cv::Mat&, const cv::Mat&)  :44, .cpp:1838-1854
//   SearchByProjection(Frame&, const vector<MapPoint*>&, th)       :61, .cpp:63-155
//   SearchByProjection(Frame&, const Frame&, th, bMono)            :78, .cpp:1506-1641
//   SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
//                                                                  :82, .cpp:1661-1790
//   SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&,
//                      vector<MapPoint*>&, int th)                 :86, .cpp:352-470
//   SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)              :104, .cpp:205-348
//   SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)           :105, .cpp:604-743
//   SearchForInitialization(Frame&, Frame&, vector<Point2f>&, vector<int>&, windowSize)
//                                                                  :108, .cpp:474-590
//   SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo)
//                                                                  :111, .cpp:755-951
//   SearchBySim3(KF1, KF2, vpMatches12, s12, R12, t12, th)         :116, .cpp:1253-1491
//   Fuse(KF, vpMapPoints, th = 3.0)                                :119, .cpp:962-1115
//   Fuse(KF, Scw, vpPoints, th, vpReplacePoint)                    :122, .cpp:1119-1249
// Fuse's searches run on the GPU, one result per MapPoint; the MapPoint
// updates (Replace / AddObservation / AddMapPoint) are then made here, on the
// host, in the reference's point order with the reference's live checks, so
// a point affected by an earlier point's update behaves as in the loop.
// The Frame / KeyFrame / MapPoint parameters are template parameters, so the
// header needs none of the reference's own headers: the members read are
// the reference's (mvKeysUn, mDescriptors, mFeatVec, mvpMapPoints, mTcw,
// GetMapPointMatches(), GetWorldPos(), ...).  One addition: the projection
// matchers need a MapPoint's raw mfMinDistance / mfMaxDistance (PredictScale,
// MapPoint.cpp:481-508, uses the raw maximum), which the reference keeps
// protected -- INTEGRATION.md adds the two public accessors GetMinDistance()
// and GetMaxDistance() to MapPoint.h.
//
// DescriptorDistance of ONE pair stays a host function (a 32-byte popcount
// is not worth a launch); the matchers compute every distance on the GPU,
// and orbgpu_hamming_pairs_device covers bulk pairs in HBM.
//
// OpenCV types come from <opencv2/core/core.hpp>, or from the header named
// by ORBGPU_CV_HEADER (the adapter tests use a small stand-in there).
// Failures throw std::runtime_error carrying orbgpu_last_error().
#ifndef ORBSLAM2_AMD_ORBMATCHER_H
#define ORBSLAM2_AMD_ORBMATCHER_H

#ifdef ORBGPU_CV_HEADER
#include ORBGPU_CV_HEADER
#else
#include <opencv2/core/core.hpp>
#endif

#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include <utility>

#include "../orbgpu.h"
#include "../orbgpu_bow.h"
#include "../orbgpu_proj.h"
#include "Device.h"

namespace orbslam2_amd {

namespace detail {
inline void check(int rc) {
    if (rc != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
}
inline orbgpu_keypoint to_kp(const cv::KeyPoint& k) {
    return orbgpu_keypoint{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave, k.class_id};
}
inline void pack_keys(const std::vector<cv::KeyPoint>& in, std::vector<orbgpu_keypoint>& out) {
    out.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) out[i] = to_kp(in[i]);
}
inline void pack_desc(const cv::Mat& m, size_t n, std::vector<unsigned char>& out) {
    if (n && (m.rows < (int)n || m.cols != 32)) throw std::invalid_argument("descriptors must be N x 32 CV_8U");
    out.resize(n * 32);
    for (size_t i = 0; i < n; ++i) std::memcpy(&out[i * 32], m.template ptr<unsigned char>((int)i), 32);
}
inline void pack_row(const cv::Mat& m, unsigned char* out32) { std::memcpy(out32, m.template ptr<unsigned char>(0), 32); }
// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>, ordered) -> CSR
template <class FV>
void pack_fv(const FV& fv, std::vector<int>& nodes, std::vector<int>& offs, std::vector<int>& feats) {
    nodes.clear();
    offs.assign(1, 0);
    feats.clear();
    for (typename FV::const_iterator it = fv.begin(); it != fv.end(); ++it) {
        nodes.push_back((int)it->first);
        for (size_t j = 0; j < it->second.size(); ++j) feats.push_back((int)it->second[j]);
        offs.push_back((int)feats.size());
    }
}
inline void mat4(const cv::Mat& T, float out[16]) {  // a 4x4 (or 3x4) CV_32F pose, row-major
    for (int i = 0; i < 16; ++i) out[i] = (i == 15) ? 1.f : 0.f;
    for (int r = 0; r < T.rows && r < 4; ++r)
        for (int c = 0; c < 4 && c < T.cols; ++c) out[4 * r + c] = T.template at<float>(r, c);
}
template <class MP>
void world_pos(MP* p, float out[3]) {
    const cv::Mat X = p->GetWorldPos();
    for (int k = 0; k < 3; ++k) out[k] = X.template at<float>(k);
}
template <class MP>
void normal(MP* p, float out[3]) {
    const cv::Mat n = p->GetNormal();
    for (int k = 0; k < 3; ++k) out[k] = n.template at<float>(k);
}
// the common target fields of a Frame or KeyFrame (Frame.h:150-200)
template <class F>
void fill_target(const F& f, int n, orbgpu_proj_target& t) {
    std::memset(&t, 0, sizeof(t));
    t.n = n;
    t.min_x = f.mnMinX;
    t.max_x = f.mnMaxX;
    t.min_y = f.mnMinY;
    t.max_y = f.mnMaxY;
    t.fx = f.fx;
    t.fy = f.fy;
    t.cx = f.cx;
    t.cy = f.cy;
    t.bf = f.mbf;
    t.b = f.mb;
    t.n_levels = f.mnScaleLevels;
    t.log_scale_factor = f.mfLogScaleFactor;
    for (int l = 0; l < (int)f.mvScaleFactors.size() && l < 16; ++l) t.scale_factors[l] = f.mvScaleFactors[l];
}
}  // namespace detail

}  // namespace orbslam2_amd

namespace ORB_SLAM2 {

class ORBmatcher {
public:
    // device (adapter-only, Device.h): the GPU the matcher's calls run on (-1: the thread's)
    ORBmatcher(float nnratio = 0.6, bool checkOri = true, int device = -1)
        : device_(device), mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    static const int TH_LOW = 50;
    static const int TH_HIGH = 100;
    static const int HISTO_LENGTH = 30;

    // Bit set count of the XOR of two 32-byte rows (ORBmatcher.cpp:1838-1854).
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
        const unsigned char* pa = a.template ptr<unsigned char>(0);
        const unsigned char* pb = b.template ptr<unsigned char>(0);
        int dist = 0;
        for (int i = 0; i < 32; i += 8) {
            uint64_t x, y;
            std::memcpy(&x, pa + i, 8);
            std::memcpy(&y, pb + i, 8);
            dist += __builtin_popcountll(x ^ y);
        }
        return dist;
    }

    // ---- SearchByProjection(F, vpMapPoints, th): local map tracking -------
    // Reads the isInFrustum() results each MapPoint carries (mbTrackInView,
    // mTrackProjX/Y/XR, mTrackViewCos, mnTrackScaleLevel); writes
    // F.mvpMapPoints[k] for every match.
    template <class FrameT, class MapPointT>
    int SearchByProjection(FrameT& F, const std::vector<MapPointT*>& vpMapPoints, const float th = 3) {
        using namespace orbslam2_amd::detail;
        const int n = (int)F.mvKeysUn.size(), np = (int)vpMapPoints.size();
        TargetBuf tb;
        target_of_frame(F, n, tb);
        std::vector<int> flags(np);
        std::vector<unsigned char> desc((size_t)np * 32);
        std::vector<float> track((size_t)np * 4);
        std::vector<int> level(np);
        for (int i = 0; i < np; ++i) {
            MapPointT* p = vpMapPoints[i];
            flags[i] = (p->mbTrackInView ? ORBGPU_PT_IN_VIEW : 0) | (!p->isBad() ? ORBGPU_PT_VALID : 0) |
                       (p->Observations() > 0 ? ORBGPU_PT_HAS_OBS : 0);
            if (!p->mbTrackInView) continue;
            pack_row(p->GetDescriptor(), &desc[(size_t)i * 32]);
            track[4 * i] = p->mTrackProjX;
            track[4 * i + 1] = p->mTrackProjY;
            track[4 * i + 2] = p->mTrackProjXR;
            track[4 * i + 3] = p->mTrackViewCos;
            level[i] = p->mnTrackScaleLevel;
        }
        orbgpu_proj_call c = make_call(ORBGPU_PROJ_LOCAL, th, tb);
        c.points.n = np;
        c.points.flags = flags.data();
        c.points.desc = desc.data();
        c.points.track = track.data();
        c.points.track_level = level.data();
        std::vector<int> match(n > 0 ? n : 1);
        int nm = run(c, match);
        for (int k = 0; k < n; ++k)
            if (match[k] >= 0) F.mvpMapPoints[k] = vpMapPoints[match[k]];
        return nm;
    }

    // ---- SearchByProjection(CurrentFrame, LastFrame, th, bMono) -----------
    template <class FrameT>
    int SearchByProjection(FrameT& CurrentFrame, const FrameT& LastFrame, const float th, const bool bMono) {
        using namespace orbslam2_amd::detail;
        const int n = (int)CurrentFrame.mvKeysUn.size(), np = LastFrame.N;
        TargetBuf tb;
        target_of_frame(CurrentFrame, n, tb);
        mat4(CurrentFrame.mTcw, tb.t.Tcw);
        std::vector<int> flags(np, 0), octave(np, 0);
        std::vector<float> pos((size_t)np * 3, 0.f), angle(np, 0.f);
        std::vector<unsigned char> desc((size_t)np * 32, 0);
        for (int i = 0; i < np; ++i) {
            auto* p = LastFrame.mvpMapPoints[i];
            if (!p || LastFrame.mvbOutlier[i]) continue;  // (:1541-1545: no isBad() test here)
            flags[i] = ORBGPU_PT_VALID | (p->Observations() > 0 ? ORBGPU_PT_HAS_OBS : 0);
            world_pos(p, &pos[3 * (size_t)i]);
            pack_row(p->GetDescriptor(), &desc[(size_t)i * 32]);
            octave[i] = LastFrame.mvKeys[i].octave;
            angle[i] = LastFrame.mvKeysUn[i].angle;
        }
        orbgpu_proj_call c = make_call(ORBGPU_PROJ_LAST_FRAME, th, tb);
        c.mono = bMono ? 1 : 0;
        mat4(LastFrame.mTcw, c.last_Tcw);
        c.points.n = np;
        c.points.flags = flags.data();
        c.points.pos = pos.data();
        c.points.desc = desc.data();
        c.points.octave = octave.data();
        c.points.angle = angle.data();
        std::vector<int> match(n > 0 ? n : 1);
        int nm = run(c, match);
        for (int k = 0; k < n; ++k) {
            if (match[k] >= 0) CurrentFrame.mvpMapPoints[k] = LastFrame.mvpMapPoints[match[k]];
            else if (match[k] == -2) CurrentFrame.mvpMapPoints[k] = nullptr;  // rotation cull
        }
        return nm;
    }

    // ---- SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist): relocalisation
    template <class FrameT, class KeyFrameT, class MapPointT>
    int SearchByProjection(FrameT& CurrentFrame, KeyFrameT* pKF, const std::set<MapPointT*>& sAlreadyFound,
                           const float th, const int ORBdist) {
        using namespace orbslam2_amd::detail;
        const int n = (int)CurrentFrame.mvKeysUn.size();
        TargetBuf tb;
        target_of_frame(CurrentFrame, n, tb);
        mat4(CurrentFrame.mTcw, tb.t.Tcw);
        const std::vector<MapPointT*> vpMPs = pKF->GetMapPointMatches();
        const int np = (int)vpMPs.size();
        PointBuf pb(np);
        for (int i = 0; i < np; ++i) {
            MapPointT* p = vpMPs[i];
            if (!p || p->isBad() || sAlreadyFound.count(p)) continue;
            pb.flags[i] = ORBGPU_PT_VALID | (p->Observations() > 0 ? ORBGPU_PT_HAS_OBS : 0);
            pb.fill(i, p);
            pb.angle[i] = pKF->mvKeysUn[i].angle;
        }
        orbgpu_proj_call c = make_call(ORBGPU_PROJ_KEYFRAME, th, tb);
        c.orb_dist = ORBdist;
        pb.attach(c.points);
        std::vector<int> match(n > 0 ? n : 1);
        int nm = run(c, match);
        for (int k = 0; k < n; ++k) {
            if (match[k] >= 0) CurrentFrame.mvpMapPoints[k] = vpMPs[match[k]];
            else if (match[k] == -2) CurrentFrame.mvpMapPoints[k] = nullptr;
        }
        return nm;
    }

    // ---- SearchByProjection(pKF, Scw, vpPoints, vpMatched, th): loop closing
    template <class KeyFrameT, class MapPointT>
    int SearchByProjection(KeyFrameT* pKF, cv::Mat Scw, const std::vector<MapPointT*>& vpPoints,
                           std::vector<MapPointT*>& vpMatched, int th) {
        using namespace orbslam2_amd::detail;
        const int n = (int)pKF->mvKeysUn.size(), np = (int)vpPoints.size();
        TargetBuf tb;
        fill_target(*pKF, n, tb.t);
        pack_keys(pKF->mvKeysUn, tb.kps);
        pack_desc(pKF->mDescriptors, n, tb.desc);
        tb.occ.assign(n > 0 ? n : 1, 0);
        for (int k = 0; k < n; ++k)
            if (vpMatched[k]) tb.occ[k] = vpMatched[k]->Observations() > 0 ? 2 : 1;
        mat4(Scw, tb.t.Tcw);
        const std::set<MapPointT*> found(vpMatched.begin(), vpMatched.end());
        PointBuf pb(np);
        for (int i = 0; i < np; ++i) {
            MapPointT* p = vpPoints[i];
            if (p->isBad() || found.count(p)) continue;
            pb.flags[i] = ORBGPU_PT_VALID | (p->Observations() > 0 ? ORBGPU_PT_HAS_OBS : 0);
            pb.fill(i, p);
            normal(p, &pb.normal[3 * (size_t)i]);
        }
        orbgpu_proj_call c = make_call(ORBGPU_PROJ_SIM3, (float)th, tb);
        pb.attach(c.points);
        std::vector<int> match(n > 0 ? n : 1);
        int nm = run(c, match);
        for (int k = 0; k < n; ++k)
            if (match[k] >= 0) vpMatched[k] = vpPoints[match[k]];
        return nm;
    }

    // ---- SearchByBoW(pKF, F, vpMapPointMatches): tracking / relocalisation
    template <class KeyFrameT, class FrameT, class MapPointT>
    int SearchByBoW(KeyFrameT* pKF, FrameT& F, std::vector<MapPointT*>& vpMapPointMatches) {
        using namespace orbslam2_amd::detail;
        const std::vector<MapPointT*> vpMapPointsKF = pKF->GetMapPointMatches();
        BowBuf a, b;
        a.set(pKF->mFeatVec, pKF->mDescriptors, (int)vpMapPointsKF.size());
        for (size_t i = 0; i < vpMapPointsKF.size(); ++i) {
            a.angle[i] = pKF->mvKeysUn[i].angle;
            a.valid[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();
        }
        b.set(F.mFeatVec, F.mDescriptors, F.N);
        for (int i = 0; i < F.N; ++i) {
            b.angle[i] = F.mvKeys[i].angle;  // (:284: F.mvKeys, not mvKeysUn)
            b.valid[i] = 1;
        }
        std::vector<int> match(F.N > 0 ? F.N : 1);
        int nm = 0;
        const orbgpu_bow_frame fa = a.frame(), fb = b.frame();
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_search_by_bow(ORBGPU_BOW_KF_F, &fa, &fb, mfNNratio, mbCheckOrientation ? 1 : 0, match.data(),
                                   &nm));
        vpMapPointMatches = std::vector<MapPointT*>(F.N, static_cast<MapPointT*>(nullptr));
        for (int i = 0; i < F.N; ++i)
            if (match[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[match[i]];
        return nm;
    }

    // ---- SearchByBoW(pKF1, pKF2, vpMatches12): loop detection ---------------
    template <class KeyFrameT, class MapPointT>
    int SearchByBoW(KeyFrameT* pKF1, KeyFrameT* pKF2, std::vector<MapPointT*>& vpMatches12) {
        using namespace orbslam2_amd::detail;
        const std::vector<MapPointT*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
        BowBuf a, b;
        a.set(pKF1->mFeatVec, pKF1->mDescriptors, (int)vp1.size());
        b.set(pKF2->mFeatVec, pKF2->mDescriptors, (int)vp2.size());
        for (size_t i = 0; i < vp1.size(); ++i) {
            a.angle[i] = pKF1->mvKeysUn[i].angle;
            a.valid[i] = vp1[i] && !vp1[i]->isBad();
        }
        for (size_t i = 0; i < vp2.size(); ++i) {
            b.angle[i] = pKF2->mvKeysUn[i].angle;
            b.valid[i] = vp2[i] && !vp2[i]->isBad();
        }
        std::vector<int> match(vp1.empty() ? 1 : vp1.size());
        int nm = 0;
        const orbgpu_bow_frame fa = a.frame(), fb = b.frame();
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_search_by_bow(ORBGPU_BOW_KF_KF, &fa, &fb, mfNNratio, mbCheckOrientation ? 1 : 0,
                                   match.data(), &nm));
        vpMatches12 = std::vector<MapPointT*>(vp1.size(), static_cast<MapPointT*>(nullptr));
        for (size_t i = 0; i < vp1.size(); ++i)
            if (match[i] >= 0) vpMatches12[i] = vp2[match[i]];
        return nm;
    }

    // ---- SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
    template <class FrameT>
    int SearchForInitialization(FrameT& F1, FrameT& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) {
        using namespace orbslam2_amd::detail;
        const size_t n1 = F1.mvKeysUn.size(), n2 = F2.mvKeysUn.size();
        if (vbPrevMatched.size() != n1) throw std::invalid_argument("vbPrevMatched size != F1 keypoints");
        std::vector<orbgpu_keypoint> k1, k2;
        std::vector<unsigned char> d1, d2;
        pack_keys(F1.mvKeysUn, k1);
        pack_keys(F2.mvKeysUn, k2);
        pack_desc(F1.mDescriptors, n1, d1);
        pack_desc(F2.mDescriptors, n2, d2);
        std::vector<float> prev(n1 * 2);
        for (size_t i = 0; i < n1; ++i) {
            prev[2 * i] = vbPrevMatched[i].x;
            prev[2 * i + 1] = vbPrevMatched[i].y;
        }
        vnMatches12.assign(n1, -1);
        const orbgpu_grid_bounds bd{F2.mnMinX, F2.mnMaxX, F2.mnMinY, F2.mnMaxY};
        const int flags = (mbCheckOrientation ? ORBGPU_MATCH_CHECK_ORI : 0) |
                          (mbAnnotatedHisto ? ORBGPU_MATCH_ANNOTATED_HISTO : 0);
        int nmatches = 0;
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_search_for_initialization(bd, k1.data(), d1.data(), (int)n1, k2.data(), d2.data(), (int)n2,
                                               prev.data(), windowSize, mfNNratio, flags, vnMatches12.data(),
                                               &nmatches));
        for (size_t i = 0; i < n1; ++i) vbPrevMatched[i] = cv::Point2f(prev[2 * i], prev[2 * i + 1]);
        return nmatches;
    }

    // ---- SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
    // LocalMapping::CreateNewMapPoints (LocalMapping.cpp:355-360)
    template <class KeyFrameT>
    int SearchForTriangulation(KeyFrameT* pKF1, KeyFrameT* pKF2, cv::Mat F12,
                               std::vector<std::pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo) {
        using namespace orbslam2_amd::detail;
        BowBuf a, b;
        const int n1 = (int)pKF1->mvKeysUn.size(), n2 = (int)pKF2->mvKeysUn.size();
        a.set(pKF1->mFeatVec, pKF1->mDescriptors, n1);
        b.set(pKF2->mFeatVec, pKF2->mDescriptors, n2);
        for (int i = 0; i < n1; ++i) {
            a.angle[i] = pKF1->mvKeysUn[i].angle;
            a.valid[i] = pKF1->GetMapPoint(i) ? 0 : 1;  // only keypoints without a MapPoint (:808-813)
        }
        for (int i = 0; i < n2; ++i) {
            b.angle[i] = pKF2->mvKeysUn[i].angle;
            b.valid[i] = pKF2->GetMapPoint(i) ? 0 : 1;
        }
        std::vector<orbgpu_keypoint> k1, k2;
        pack_keys(pKF1->mvKeysUn, k1);
        pack_keys(pKF2->mvKeysUn, k2);
        if (k1.empty()) k1.resize(1);
        if (k2.empty()) k2.resize(1);
        orbgpu_triangulation_pair P;
        std::memset(&P, 0, sizeof(P));
        P.kf1 = a.frame();
        P.kf2 = b.frame();
        P.kps1 = k1.data();
        P.kps2 = k2.data();
        P.u_right1 = (int)pKF1->mvuRight.size() >= n1 && n1 ? pKF1->mvuRight.data() : nullptr;
        P.u_right2 = (int)pKF2->mvuRight.size() >= n2 && n2 ? pKF2->mvuRight.data() : nullptr;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) P.F12[3 * r + c] = F12.template at<float>(r, c);
        const cv::Mat Cw = pKF1->GetCameraCenter(), R2w = pKF2->GetRotation(), t2w = pKF2->GetTranslation();
        for (int r = 0; r < 3; ++r) {
            P.Cw1[r] = Cw.template at<float>(r);
            for (int c = 0; c < 3; ++c) P.T2w[4 * r + c] = R2w.template at<float>(r, c);
            P.T2w[4 * r + 3] = t2w.template at<float>(r);
        }
        P.fx2 = pKF2->fx;
        P.fy2 = pKF2->fy;
        P.cx2 = pKF2->cx;
        P.cy2 = pKF2->cy;
        for (int l = 0; l < (int)pKF2->mvScaleFactors.size() && l < 16; ++l) P.scale_factors2[l] = pKF2->mvScaleFactors[l];
        for (int l = 0; l < (int)pKF2->mvLevelSigma2.size() && l < 16; ++l) P.level_sigma2_2[l] = pKF2->mvLevelSigma2[l];
        P.only_stereo = bOnlyStereo ? 1 : 0;
        std::vector<int> m12(n1 > 0 ? n1 : 1);
        int nm = 0;
        const orbslam2_amd::DeviceGuard device_guard(device_);
        check(orbgpu_search_for_triangulation(&P, mbCheckOrientation ? 1 : 0, m12.data(), &nm));
        vMatchedPairs.clear();
        vMatchedPairs.reserve(nm);
        for (int i = 0; i < n1; ++i)
            if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
        return nm;
    }

    // ---- SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) ---------
    // LoopClosing::ComputeSim3 (LoopClosing.cpp:386)
    template <class KeyFrameT, class MapPointT>
    int SearchBySim3(KeyFrameT* pKF1, KeyFrameT* pKF2, std::vector<MapPointT*>& vpMatches12, const float& s12,
                     const cv::Mat& R12, const cv::Mat& t12, const float th) {
        using namespace orbslam2_amd::detail;
        const std::vector<MapPointT*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
        const int N1 = (int)vp1.size(), N2 = (int)vp2.size();
        std::vector<char> already1(N1, 0), already2(N2, 0);  // vbAlreadyMatched1/2 (:1282-1296)
        for (int i = 0; i < N1; ++i)
            if (MapPointT* pMP = vpMatches12[i]) {
                already1[i] = 1;
                const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
                if (idx2 >= 0 && idx2 < N2) already2[idx2] = 1;
            }
        TargetBuf t1, t2;
        keyframe_target(*pKF1, t1);
        keyframe_target(*pKF2, t2);
        PointBuf p1(N1), p2(N2);
        for (int i = 0; i < N1; ++i) {
            MapPointT* p = vp1[i];
            if (!p || already1[i] || p->isBad()) continue;
            p1.flags[i] = ORBGPU_PT_VALID;
            p1.fill(i, p);
        }
        for (int i = 0; i < N2; ++i) {
            MapPointT* p = vp2[i];
            if (!p || already2[i] || p->isBad()) continue;
            p2.flags[i] = ORBGPU_PT_VALID;
            p2.fill(i, p);
        }
        orbgpu_sim3_search S;
        std::memset(&S, 0, sizeof(S));
        S.kf1 = attach_target(t1);
        S.kf2 = attach_target(t2);
        p1.attach(S.pts1);
        p2.attach(S.pts2);
        S.s12 = s12;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) S.R12[3 * r + c] = R12.template at<float>(r, c);
            S.t12[r] = t12.template at<float>(r);
        }
        S.th = th;
        std::vector<int> m12(N1 > 0 ? N1 : 1);
        int nfound = 0;
        check(orbgpu_search_by_sim3(&S, m12.data(), &nfound));
        for (int i = 0; i < N1; ++i)
            if (m12[i] >= 0) vpMatches12[i] = vp2[m12[i]];
        return nfound;
    }

    // ---- Fuse(pKF, vpMapPoints, th): LocalMapping::SearchInNeighbors -------
    template <class KeyFrameT, class MapPointT>
    int Fuse(KeyFrameT* pKF, const std::vector<MapPointT*>& vpMapPoints, const float th = 3.0) {
        using namespace orbslam2_amd::detail;
        TargetBuf tb;
        keyframe_target(*pKF, tb);
        const int np = (int)vpMapPoints.size();
        PointBuf pb(np);
        for (int i = 0; i < np; ++i) {
            MapPointT* p = vpMapPoints[i];
            if (!p || p->isBad() || p->IsInKeyFrame(pKF)) continue;
            pb.flags[i] = ORBGPU_PT_VALID;
            pb.fill(i, p);
            normal(p, &pb.normal[3 * (size_t)i]);
        }
        const std::vector<int> best = per_point(ORBGPU_PROJ_FUSE, th, tb, pb);
        int nFused = 0;
        for (int i = 0; i < np; ++i) {  // the reference's updates, in its order (:1091-1111)
            MapPointT* pMP = vpMapPoints[i];
            if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF) || best[i] < 0) continue;
            MapPointT* pMPinKF = pKF->GetMapPoint(best[i]);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) {
                    if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                    else pMPinKF->Replace(pMP);
                }
            } else {
                pMP->AddObservation(pKF, best[i]);
                pKF->AddMapPoint(pMP, best[i]);
            }
            nFused++;
        }
        return nFused;
    }

    // ---- Fuse(pKF, Scw, vpPoints, th, vpReplacePoint): LoopClosing::SearchAndFuse
    template <class KeyFrameT, class MapPointT>
    int Fuse(KeyFrameT* pKF, cv::Mat Scw, const std::vector<MapPointT*>& vpPoints, float th,
             std::vector<MapPointT*>& vpReplacePoint) {
        using namespace orbslam2_amd::detail;
        TargetBuf tb;
        keyframe_target(*pKF, tb);
        mat4(Scw, tb.t.Tcw);
        const std::set<MapPointT*> spAlreadyFound = pKF->GetMapPoints();
        const int np = (int)vpPoints.size();
        PointBuf pb(np);
        for (int i = 0; i < np; ++i) {
            MapPointT* p = vpPoints[i];
            if (p->isBad() || spAlreadyFound.count(p)) continue;
            pb.flags[i] = ORBGPU_PT_VALID;
            pb.fill(i, p);
            normal(p, &pb.normal[3 * (size_t)i]);
        }
        const std::vector<int> best = per_point(ORBGPU_PROJ_FUSE_SIM3, th, tb, pb);
        int nFused = 0;
        for (int i = 0; i < np; ++i) {  // :1228-1245
            MapPointT* pMP = vpPoints[i];
            if (pMP->isBad() || spAlreadyFound.count(pMP) || best[i] < 0) continue;
            MapPointT* pMPinKF = pKF->GetMapPoint(best[i]);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
            } else {
                pMP->AddObservation(pKF, best[i]);
                pKF->AddMapPoint(pMP, best[i]);
            }
            nFused++;
        }
        return nFused;
    }

    // Extension (not in the reference): the annotated tree's rotation-bin
    // factor 1/HISTO_LENGTH in SearchForInitialization.
    bool mbAnnotatedHisto = false;

protected:
    int device_ = -1;
    float mfNNratio;
    bool mbCheckOrientation;

private:
    struct TargetBuf {
        orbgpu_proj_target t;
        std::vector<orbgpu_keypoint> kps;
        std::vector<unsigned char> desc, occ;
        std::vector<float> ur;
    };
    struct PointBuf {
        std::vector<int> flags;
        std::vector<float> pos, normal, min_dist, max_dist, angle;
        std::vector<unsigned char> desc;
        explicit PointBuf(int np)
            : flags(np, 0), pos((size_t)np * 3, 0.f), normal((size_t)np * 3, 0.f), min_dist(np, 0.f),
              max_dist(np, 0.f), angle(np, 0.f), desc((size_t)np * 32, 0) {}
        template <class MP>
        void fill(int i, MP* p) {
            orbslam2_amd::detail::world_pos(p, &pos[3 * (size_t)i]);
            orbslam2_amd::detail::pack_row(p->GetDescriptor(), &desc[(size_t)i * 32]);
            min_dist[i] = p->GetMinDistance();  // raw mfMinDistance
            max_dist[i] = p->GetMaxDistance();  // raw mfMaxDistance
        }
        void attach(orbgpu_proj_points& P) {
            P.n = (int)flags.size();
            P.flags = flags.data();
            P.pos = pos.data();
            P.normal = normal.data();
            P.desc = desc.data();
            P.min_dist = min_dist.data();
            P.max_dist = max_dist.data();
            P.angle = angle.data();
        }
    };
    struct BowBuf {
        std::vector<int> nodes, offs, feats;
        std::vector<unsigned char> desc, valid;
        std::vector<float> angle;
        int n = 0;
        template <class FV>
        void set(const FV& fv, const cv::Mat& d, int n_) {
            n = n_;
            orbslam2_amd::detail::pack_fv(fv, nodes, offs, feats);
            orbslam2_amd::detail::pack_desc(d, (size_t)n, desc);
            angle.assign(n > 0 ? n : 1, 0.f);
            valid.assign(n > 0 ? n : 1, 0);
            if (desc.empty()) desc.assign(32, 0);
            if (feats.empty()) feats.assign(1, 0);
        }
        orbgpu_bow_frame frame() const {
            return orbgpu_bow_frame{n, (int)nodes.size(), nodes.data(), offs.data(), feats.data(), desc.data(),
                                    angle.data(), valid.data()};
        }
    };

    template <class FrameT>
    static void target_of_frame(const FrameT& F, int n, TargetBuf& tb) {
        using namespace orbslam2_amd::detail;
        fill_target(F, n, tb.t);
        pack_keys(F.mvKeysUn, tb.kps);
        pack_desc(F.mDescriptors, (size_t)n, tb.desc);
        tb.occ.assign(n > 0 ? n : 1, 0);
        tb.ur.assign(n > 0 ? n : 1, -1.f);
        for (int k = 0; k < n; ++k) {
            if (F.mvpMapPoints[k]) tb.occ[k] = F.mvpMapPoints[k]->Observations() > 0 ? 2 : 1;
            if (k < (int)F.mvuRight.size()) tb.ur[k] = F.mvuRight[k];
        }
    }

    // a KeyFrame as a projection target: mvKeysUn, descriptors, mvuRight,
    // pose [GetRotation() | GetTranslation()]
    template <class KeyFrameT>
    static void keyframe_target(KeyFrameT& KF, TargetBuf& tb) {
        using namespace orbslam2_amd::detail;
        const int n = (int)KF.mvKeysUn.size();
        fill_target(KF, n, tb.t);
        pack_keys(KF.mvKeysUn, tb.kps);
        pack_desc(KF.mDescriptors, (size_t)n, tb.desc);
        tb.occ.assign(n > 0 ? n : 1, 0);
        tb.ur.assign(n > 0 ? n : 1, -1.f);
        for (int k = 0; k < n && k < (int)KF.mvuRight.size(); ++k) tb.ur[k] = KF.mvuRight[k];
        const cv::Mat R = KF.GetRotation(), t = KF.GetTranslation();
        for (int i = 0; i < 16; ++i) tb.t.Tcw[i] = (i == 15) ? 1.f : 0.f;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) tb.t.Tcw[4 * r + c] = R.template at<float>(r, c);
            tb.t.Tcw[4 * r + 3] = t.template at<float>(r);
        }
    }

    static orbgpu_proj_target attach_target(TargetBuf& tb) {
        orbgpu_proj_target t = tb.t;
        if (tb.kps.empty()) tb.kps.resize(1);
        if (tb.desc.empty()) tb.desc.assign(32, 0);
        t.kps = tb.kps.data();
        t.desc = tb.desc.data();
        t.occupied = nullptr;
        t.u_right = tb.ur.data();
        return t;
    }

    // one per-point search (FUSE / FUSE_SIM3): best keypoint per point or -1
    std::vector<int> per_point(int variant, float th, TargetBuf& tb, PointBuf& pb) const {
        orbgpu_proj_call c = make_call(variant, th, tb);
        c.target.occupied = nullptr;
        pb.attach(c.points);
        std::vector<int> best(pb.flags.empty() ? 1 : pb.flags.size());
        run(c, best);
        best.resize(pb.flags.size());
        return best;
    }

    orbgpu_proj_call make_call(int variant, float th, TargetBuf& tb) const {
        orbgpu_proj_call c;
        std::memset(&c, 0, sizeof(c));
        c.variant = variant;
        c.check_ori = mbCheckOrientation ? 1 : 0;
        c.nnratio = mfNNratio;
        c.th = th;
        c.target = tb.t;
        if (tb.kps.empty()) tb.kps.resize(1);
        if (tb.desc.empty()) tb.desc.assign(32, 0);
        c.target.kps = tb.kps.data();
        c.target.desc = tb.desc.data();
        c.target.occupied = tb.occ.data();
        c.target.u_right = tb.ur.empty() ? nullptr : tb.ur.data();
        return c;
    }

    int run(const orbgpu_proj_call& c, std::vector<int>& match) const {
        int nm = 0;
        const orbslam2_amd::DeviceGuard device_guard(device_);
        orbslam2_amd::detail::check(orbgpu_search_by_projection(&c, match.data(), &nm));
        return nm;
    }
};

}  // namespace ORB_SLAM2

namespace orbslam2_amd {
// Round-1 free-function form, kept for existing callers.
template <class FrameT>
int SearchForInitialization(float nnratio, bool checkOri, FrameT& F1, FrameT& F2,
                            std::vector<cv::Point2f>& vbPrevMatched, std::vector<int>& vnMatches12,
                            int windowSize = 10, bool annotatedHisto = false) {
    ORB_SLAM2::ORBmatcher m(nnratio, checkOri);
    m.mbAnnotatedHisto = annotatedHisto;
    return m.SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize);
}
}  // namespace orbslam2_amd

#endif
