// proj_ref.cpp -- C++ restatement of the two ORBmatcher::SearchByProjection
// overloads Tracking calls on every frame, with Frame::GetFeaturesInArea:
//   LOCAL      SearchByProjection(Frame&, vector<MapPoint*>&, th)
//              (ORBmatcher.cpp:63-155; Tracking::SearchLocalPoints,
//              Tracking.cpp:1560), on the isInFrustum track fields;
//   LAST_FRAME SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
//              th, bMono) (ORBmatcher.cpp:1506-1641;
//              Tracking::TrackWithMotionModel, Tracking.cpp:1152-1160).
//
// TEST INFRASTRUCTURE ONLY.  It follows oracle/proj_ref.py line for line in
// float arithmetic (float32 steps, cv::Mat products accumulated in double,
// cvRound as floor(|v| + 0.5) with the sign), so its matches equal the
// Python oracle's bit for bit (tests/test_oracle_proj_cpp.py); it exists so
// the drop-in latency table times compiled code on the CPU side
// (bench.py DropIn.cpu_oracle), not Python.  Parity unpinned against the
// reference binary (OpenCV 2.4 absent), as proj_ref.py.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int kGC = 64, kGR = 48, kHL = 30, kThHigh = 100;
constexpr int kValid = 1, kHasObs = 2, kInView = 4;
constexpr int kLocal = 0, kLastFrame = 2;

struct Kp {  // cv::KeyPoint layout (28 B)
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

float dotd3(const float* a, const float* x) {  // cv::Mat float product, double accumulation
    return (float)((double)a[0] * (double)x[0] + (double)a[1] * (double)x[1] + (double)a[2] * (double)x[2]);
}

int c_round(double v) { return (int)std::copysign(std::floor(std::fabs(v) + 0.5), v); }

int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int k = 0; k < 32; k += 8) {
        uint64_t x, y;
        std::memcpy(&x, a + k, 8);
        std::memcpy(&y, b + k, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}

struct Grid {  // Frame::AssignFeaturesToGrid / GetFeaturesInArea (Frame.cpp:241-259, 379-443)
    const Kp* k;
    float mnx, mny, invW, invH;
    std::vector<int> cells[kGC][kGR];
    Grid(const Kp* kps, int n, const float* b) : k(kps), mnx(b[0]), mny(b[2]) {
        invW = (float)kGC / (b[1] - b[0]);
        invH = (float)kGR / (b[3] - b[2]);
        for (int i = 0; i < n; ++i) {
            const int px = c_round((double)((k[i].x - mnx) * invW));
            const int py = c_round((double)((k[i].y - mny) * invH));
            if (px >= 0 && px < kGC && py >= 0 && py < kGR) cells[px][py].push_back(i);
        }
    }
    void area(float x, float y, float r, int min_level, int max_level, std::vector<int>& out) const {
        out.clear();
        const int cx0 = std::max(0, (int)std::floor((double)(((x - mnx) - r) * invW)));
        if (cx0 >= kGC) return;
        const int cx1 = std::min(kGC - 1, (int)std::ceil((double)(((x - mnx) + r) * invW)));
        if (cx1 < 0) return;
        const int cy0 = std::max(0, (int)std::floor((double)(((y - mny) - r) * invH)));
        if (cy0 >= kGR) return;
        const int cy1 = std::min(kGR - 1, (int)std::ceil((double)(((y - mny) + r) * invH)));
        if (cy1 < 0) return;
        const bool check = min_level > 0 || max_level >= 0;
        for (int ix = cx0; ix <= cx1; ++ix)
            for (int iy = cy0; iy <= cy1; ++iy)
                for (int i : cells[ix][iy]) {
                    const int o = k[i].octave;
                    if (check) {
                        if (o < min_level) continue;
                        if (max_level >= 0 && o > max_level) continue;
                    }
                    if (std::fabs(k[i].x - x) < r && std::fabs(k[i].y - y) < r) out.push_back(i);
                }
    }
};

}  // namespace

extern "C" {

// tgt: kps[n], desc[n][32], u_right[n] (nullable), occupied[n] (nullable, 0 /
// 1 / 2), bounds {min_x, max_x, min_y, max_y}, cam {fx, fy, cx, cy, bf, b},
// scale_factors[8], Tcw[16] (row-major 4x4).  pts: flags, pos[3], desc[32],
// track[4] (u, v, u_right, viewing cos; LOCAL), track_level (LOCAL), octave
// and angle (LAST_FRAME).  last_Tcw: LastFrame.mTcw (LAST_FRAME).  match[n]:
// point index, -1 untouched, -2 set to NULL by the rotation cull.  Returns
// nmatches, or -1 for an unsupported variant.
int orbref_search_by_projection(int variant, const Kp* kps, const uint8_t* tdesc, int n, const float* u_right,
                                const uint8_t* occupied, const float* bounds, const float* cam,
                                const float* scale_factors, const float* Tcw, int npts, const int* flags,
                                const float* pos, const uint8_t* pdesc, const float* track, const int* track_level,
                                const int* octave, const float* angle, const float* last_Tcw, float th,
                                float nnratio, int check_ori, int mono, int* match) {
    if (variant != kLocal && variant != kLastFrame) return -1;
    Grid grid(kps, n, bounds);
    std::vector<uint8_t> occ(n, 0);
    if (occupied) occ.assign(occupied, occupied + n);
    for (int i = 0; i < n; ++i) match[i] = -1;
    std::vector<int> hist[kHL];
    const float factor = (float)kHL / 360.0f;
    const float fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3], bf = cam[4], b = cam[5];
    bool forward = false, backward = false;
    if (variant == kLastFrame) {  // ORBmatcher.cpp:1519-1527
        float O[3];
        for (int j = 0; j < 3; ++j) {
            const float col[3] = {Tcw[j], Tcw[4 + j], Tcw[8 + j]};
            const float t[3] = {Tcw[3], Tcw[7], Tcw[11]};
            O[j] = -dotd3(col, t);
        }
        const float tlc_z = dotd3(last_Tcw + 8, O) + last_Tcw[11];
        forward = tlc_z > b && !mono;
        backward = -tlc_z > b && !mono;
    }
    int nm = 0;
    std::vector<int> cands;
    cands.reserve(256);
    for (int ip = 0; ip < npts; ++ip) {
        const int fl = flags[ip];
        if (!(fl & kValid)) continue;
        float ur = 0.f, srad = 0.f;
        if (variant == kLocal) {
            if (!(fl & kInView)) continue;
            const int lvl = track_level[ip];
            const float* tr = track + 4 * ip;
            float r = (double)tr[3] > 0.998 ? 2.5f : 4.0f;
            if (th != 1.0f) r = r * th;
            const float rad = r * scale_factors[lvl];
            grid.area(tr[0], tr[1], rad, lvl - 1, lvl, cands);
            ur = tr[2];
            srad = rad;
        } else {
            const float* X = pos + 3 * ip;
            float pc[3];
            for (int i = 0; i < 3; ++i) pc[i] = dotd3(Tcw + 4 * i, X) + Tcw[4 * i + 3];
            const float invzc = (float)(1.0 / (double)pc[2]);
            if (invzc < 0) continue;
            const float u = (fx * pc[0]) * invzc + cx;
            const float v = (fy * pc[1]) * invzc + cy;
            if (u < bounds[0] || u > bounds[1] || v < bounds[2] || v > bounds[3]) continue;
            const int o = octave[ip];
            const float rad = th * scale_factors[o];
            if (forward)
                grid.area(u, v, rad, o, -1, cands);
            else if (backward)
                grid.area(u, v, rad, 0, o, cands);
            else
                grid.area(u, v, rad, o - 1, o + 1, cands);
            ur = u - bf * invzc;
            srad = rad;
        }
        if (cands.empty()) continue;
        const uint8_t* d = pdesc + 32 * ip;
        int best = 256, best_i = -1, best_l = -1, best2 = 256, best_l2 = -1;
        for (int i : cands) {
            if (occ[i] == 2) continue;
            if (u_right && u_right[i] > 0 && std::fabs(ur - u_right[i]) > srad) continue;
            const int dist = hamming(d, tdesc + 32 * i);
            if (dist < best) {
                best2 = best;
                best_l2 = best_l;
                best = dist;
                best_i = i;
                best_l = kps[i].octave;
            } else if (dist < best2) {
                best2 = dist;
                best_l2 = kps[i].octave;
            }
        }
        if (!(best <= kThHigh)) continue;
        if (variant == kLocal && best_l == best_l2 && (float)best > nnratio * (float)best2) continue;
        match[best_i] = ip;
        occ[best_i] = (fl & kHasObs) ? 2 : 1;
        ++nm;
        if (check_ori && variant == kLastFrame) {
            float rot = angle[ip] - kps[best_i].angle;
            if (rot < 0.0f) rot = rot + 360.0f;
            int bin = c_round((double)(rot * factor));
            if (bin == kHL) bin = 0;
            hist[bin].push_back(best_i);
        }
    }
    if (check_ori && variant == kLastFrame) {  // ComputeThreeMaxima (ORBmatcher.cpp:1792-1833) and the cull
        int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
        for (int i = 0; i < kHL; ++i) {
            const int s = (int)hist[i].size();
            if (s > m1) {
                m3 = m2; m2 = m1; m1 = s;
                i3 = i2; i2 = i1; i1 = i;
            } else if (s > m2) {
                m3 = m2; m2 = s;
                i3 = i2; i2 = i;
            } else if (s > m3) {
                m3 = s;
                i3 = i;
            }
        }
        if ((float)m2 < 0.1f * (float)m1) {
            i2 = -1;
            i3 = -1;
        } else if ((float)m3 < 0.1f * (float)m1) {
            i3 = -1;
        }
        for (int i = 0; i < kHL; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int slot : hist[i]) {
                match[slot] = -2;
                --nm;
            }
        }
    }
    return nm;
}

}  // extern "C"
