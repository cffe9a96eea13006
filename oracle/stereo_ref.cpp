/*
 * stereo_ref.cpp -- C++ restatement of Frame::ComputeStereoMatches (TEST
 * INFRASTRUCTURE ONLY: the compiled twin of oracle/stereo_ref.py, used by
 * bench.py's stereo cpu_baseline legs and by tests/; the product never
 * links it).  F = /root/reference/ORB-SLAM2/src/Frame.cpp.
 *
 * The spec is stereo_ref.py's, statement for statement, in
 * float with -ffp-contract=off: row bands of the right keypoints (F:555-576),
 * the best Hamming distance within the disparity range and octave window
 * (F:597-642), the 11x11 SAD over 11 shifts on the two pyramid levels
 * (F:645-700), the parabola fit (F:702-716), depth (F:718-729) and the
 * median cut (F:734-747).  tests/test_stereo.py checks it against
 * stereo_ref.py bit for bit.
 */
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "orbref.h"

namespace {

int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

float c_roundf(float v) { return std::round(v); }  // std::round(float): half away from zero

}  // namespace

extern "C" void orbref_stereo_matches(const orbref_extractor* exL, const orbref_extractor* exR,
                                      const orbref_kp* kpsL, const uint8_t* descL, int nL, const orbref_kp* kpsR,
                                      const uint8_t* descR, int nR, float bf, float min_z, float* uright,
                                      float* depth) {
    const int TH_HIGH = 100, TH_LOW = 50;
    const int nlev = orbref_level_count(exL);
    std::vector<float> scale(nlev), inv(nlev), s2(nlev), is2(nlev);
    orbref_scale_factors(exL, scale.data(), inv.data(), s2.data(), is2.data());
    for (int i = 0; i < nL; ++i) { uright[i] = -1.0f; depth[i] = -1.0f; }
    int w0, h0;
    orbref_level_ptr(exL, 0, &w0, &h0);
    const int n_rows = h0;
    const int th_orb = (TH_HIGH + TH_LOW) / 2;  // F:545
    std::vector<std::vector<int>> rows(n_rows);  // F:555-576
    for (int iR = 0; iR < nR; ++iR) {
        const float ky = kpsR[iR].y;
        const float r = 2.0f * scale[kpsR[iR].octave];
        const int maxr = (int)std::ceil(ky + r);
        const int minr = (int)std::floor(ky - r);
        for (int yi = minr; yi <= maxr; ++yi)
            if (yi >= 0 && yi < n_rows) rows[yi].push_back(iR);
    }
    const float min_d = 0.0f;
    const float max_d = bf / min_z;  // F:581 (mb = 0 at call time: +inf)
    std::vector<std::pair<int, int>> dist_idx;
    for (int iL = 0; iL < nL; ++iL) {
        const int lvl = kpsL[iL].octave;
        const float vL = kpsL[iL].y, uL = kpsL[iL].x;
        if ((int)vL >= n_rows) continue;
        const std::vector<int>& cand = rows[(int)vL];
        if (cand.empty()) continue;
        const float min_u = uL - max_d;
        const float max_u = uL - min_d;
        if (max_u < 0) continue;
        int best = TH_HIGH, best_r = 0;
        for (int iR : cand) {  // F:618-640
            const int o = kpsR[iR].octave;
            if (o < lvl - 1 || o > lvl + 1) continue;
            const float uR = kpsR[iR].x;
            if (uR >= min_u && uR <= max_u) {
                const int d = hamming32(descL + 32 * iL, descR + 32 * iR);
                if (d < best) { best = d; best_r = iR; }
            }
        }
        if (best >= th_orb) continue;
        const float uR0 = kpsR[best_r].x;
        const float sf = inv[lvl];
        const float su = c_roundf(uL * sf);
        const float sv = c_roundf(vL * sf);
        const float sr = c_roundf(uR0 * sf);
        const int w = 5, L = 5;
        int lw, lh, rw, rh;
        const uint8_t* IL = orbref_level_ptr(exL, lvl, &lw, &lh);
        const uint8_t* IR = orbref_level_ptr(exR, lvl, &rw, &rh);
        const int r0 = (int)sv - w, c0 = (int)su - w;
        if (r0 < 0 || r0 + 2 * w + 1 > lh || c0 < 0 || c0 + 2 * w + 1 > lw) continue;
        const float iniu = sr + L - w;
        const float endu = sr + L + w + 1;
        if (iniu < 0 || endu >= rw) continue;  // F:668-671
        if ((int)sr - L - w < 0 || r0 + 2 * w + 1 > rh) continue;  // spec: the IR window would leave the level
        const int cL = IL[(size_t)(r0 + w) * lw + c0 + w];
        int best_sad = INT_MAX, best_inc = 0;
        float dists[11];
        for (int inc = -L; inc <= L; ++inc) {
            const int cr = (int)sr + inc - w;
            const int cR = IR[(size_t)(r0 + w) * rw + cr + w];
            long sad = 0;
            for (int y = 0; y < 11; ++y)
                for (int x = 0; x < 11; ++x) {
                    const int a = IL[(size_t)(r0 + y) * lw + c0 + x] - cL;
                    const int b = IR[(size_t)(r0 + y) * rw + cr + x] - cR;
                    sad += std::abs(a - b);
                }
            if (sad < best_sad) { best_sad = (int)sad; best_inc = inc; }
            dists[L + inc] = (float)sad;
        }
        if (best_inc == -L || best_inc == L) continue;
        const float d1 = dists[L + best_inc - 1], d2 = dists[L + best_inc], d3 = dists[L + best_inc + 1];
        const float delta = (d1 - d3) / (2.0f * ((d1 + d3) - 2.0f * d2));
        if (delta < -1 || delta > 1) continue;
        float best_uR = scale[lvl] * ((sr + (float)best_inc) + delta);
        float disp = uL - best_uR;
        if (disp >= min_d && disp < max_d) {
            if (disp <= 0) {
                disp = 0.01f;
                best_uR = (float)((double)uL - 0.01);
            }
            depth[iL] = bf / disp;
            uright[iL] = best_uR;
            dist_idx.emplace_back(best_sad, iL);
        }
    }
    if (!dist_idx.empty()) {  // F:734-747
        std::sort(dist_idx.begin(), dist_idx.end());
        const float median = (float)dist_idx[dist_idx.size() / 2].first;
        const float th = (1.5f * 1.4f) * median;
        for (int i = (int)dist_idx.size() - 1; i >= 0; --i) {
            if ((float)dist_idx[i].first < th) break;
            uright[dist_idx[i].second] = -1.0f;
            depth[dist_idx[i].second] = -1.0f;
        }
    }
}
