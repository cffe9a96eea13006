// proj.hip -- the projection matchers (include/orbgpu_proj.h):
// Frame::isInFrustum, the four ORBmatcher::SearchByProjection overloads and
// the per-point radius searches of ORBmatcher::Fuse (both overloads) and
// SearchBySim3 (one direction per call).
//
// One 1024-thread block per call (proj_kernel, below): the target's feature
// grid in LDS, every point's projection and candidate list built by 15
// waves in parallel (4 lanes per point), the reference's sequential point
// walk (an assignment hides a keypoint from later points) replayed by one
// wave from those lists, then the rotation-consistency cull.  Candidate keys (Hamming distance <<
// 20 | grid position) reproduce the reference's first-best-in-order choice.
#include "../../include/orbgpu_proj.h"
#include "proj_kernels.h"
#include "device_state.h"
#include "group_sum.h"

namespace orbgpu {

namespace {

constexpr int kMaxKps = 4096;
constexpr int kGC = 64, kGR = 48, kCells = kGC * kGR;
constexpr int kHL = 30, kThLow = 50, kThHigh = 100;

__device__ inline float dotd3(const float* a, const float* x) {  // cv::Mat float product, double accumulation
    return (float)((double)a[0] * (double)x[0] + (double)a[1] * (double)x[1] + (double)a[2] * (double)x[2]);
}

// Rcw*x + tcw with R = T[0..2][0..2], t = T[..][3] (row-major 4x4)
__device__ inline void transform(const float* T, const float* x, float* y) {
    for (int i = 0; i < 3; ++i) {
        const float r[3] = {T[4 * i], T[4 * i + 1], T[4 * i + 2]};
        y[i] = dotd3(r, x) + T[4 * i + 3];
    }
}

// -Rcw^T * tcw
__device__ inline void camera_center(const float* T, float* O) {
    for (int j = 0; j < 3; ++j) {
        const float c[3] = {T[j], T[4 + j], T[8 + j]};
        const float t[3] = {T[3], T[7], T[11]};
        O[j] = -dotd3(c, t);
    }
}

// MapPoint::PredictScale (MapPoint.cpp:481-508)
__device__ inline int predict_scale(float max_dist, float dist, const orbgpu_proj_target& T) {
    const float ratio = max_dist / dist;
    const float l = (float)log((double)ratio);
    int s = (int)ceilf(l / T.log_scale_factor);
    if (s < 0) s = 0;
    else if (s >= T.n_levels) s = T.n_levels - 1;
    return s;
}

// one point's search parameters after projection
struct Query {
    bool ok;
    int flags;           // the point's ORBGPU_PT_* flags
    float angle;         // its descriptor angle (rotation-checked variants)
    float u, v, r;       // window centre and half-size
    int min_level, max_level;
    float ur;            // stereo: projected right coordinate (LOCAL, LAST_FRAME)
    float stereo_r;      // stereo tolerance
    bool stereo;
    bool chi2;               // FUSE: the reprojection chi-square test (ORBmatcher.cpp:1053-1078)
    int level_lo, level_hi;  // SIM3 / FUSE* / SIM3_DIR: keypoint level window applied after the area query
};

// variants that report one result per point (best keypoint in the window,
// no hidden set, no sequential walk)
__device__ inline bool per_point(int variant) { return variant >= ORBGPU_PROJ_FUSE; }

// Per-call pose quantities shared by every point of the call.
struct CallPose {
    float O[3];
    float Rs[16];  // SIM3: [Rcw | tcw] after removing the scale
    bool forward, backward;
};

__device__ __forceinline__ CallPose call_pose(const orbgpu_proj_call& C) {
    CallPose cp{};
    const orbgpu_proj_target& T = C.target;
    const float* Tcw = T.Tcw;
    if (C.variant == ORBGPU_PROJ_SIM3 || C.variant == ORBGPU_PROJ_FUSE_SIM3) {  // ORBmatcher.cpp:361-371, :1129-1133
        const float row0[3] = {Tcw[0], Tcw[1], Tcw[2]};
        const float scw = (float)sqrt((double)row0[0] * row0[0] + (double)row0[1] * row0[1] + (double)row0[2] * row0[2]);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) cp.Rs[4 * i + j] = Tcw[4 * i + j] / scw;
            cp.Rs[4 * i + 3] = Tcw[4 * i + 3] / scw;
        }
        camera_center(cp.Rs, cp.O);
    } else if (C.variant == ORBGPU_PROJ_FUSE) {  // pKF->GetCameraCenter() (KeyFrame::SetPose: Ow = -Rcw^T tcw)
        camera_center(Tcw, cp.O);
    } else if (C.variant == ORBGPU_PROJ_LAST_FRAME || C.variant == ORBGPU_PROJ_KEYFRAME) {
        float twc[3];
        camera_center(Tcw, twc);  // twc = -Rcw^T tcw (= Ow)
        for (int j = 0; j < 3; ++j) cp.O[j] = twc[j];
        if (C.variant == ORBGPU_PROJ_LAST_FRAME) {  // ORBmatcher.cpp:1521-1527
            const float* L = C.last_Tcw;
            const float r2[3] = {L[8], L[9], L[10]};
            const float tlc_z = dotd3(r2, twc) + L[11];
            if (!C.mono) {
                cp.forward = tlc_z > T.b;
                cp.backward = -tlc_z > T.b;
            }
        }
    }
    return cp;
}

// The reference's per-point projection and window for the call's variant.
// Every point field the variant reads is loaded up front, independent of the
// flags, so a point costs one memory latency; sf = the target's scale
// factors (16 entries, in LDS).
__device__ __forceinline__ Query make_query(const orbgpu_proj_call& C, const CallPose& cp, const float* sf, int ip) {
    const orbgpu_proj_target& T = C.target;
    const orbgpu_proj_points& P = C.points;
    const int variant = C.variant;
    const int fl = P.flags[ip];
    float X[3] = {0.f, 0.f, 0.f}, tr[4] = {0.f, 0.f, 0.f, 0.f}, Pn[3] = {0.f, 0.f, 0.f};
    float maxd0 = 0.f, mind0 = 0.f;
    int lv = 0;
    if (variant == ORBGPU_PROJ_LOCAL) {
        for (int k = 0; k < 4; ++k) tr[k] = P.track[4 * ip + k];
        lv = P.track_level[ip];
    } else {
        for (int k = 0; k < 3; ++k) X[k] = P.pos[3 * ip + k];
        if (variant != ORBGPU_PROJ_LAST_FRAME) {
            maxd0 = P.max_dist[ip];
            mind0 = P.min_dist[ip];
        }
        if (variant == ORBGPU_PROJ_SIM3 || variant == ORBGPU_PROJ_FUSE || variant == ORBGPU_PROJ_FUSE_SIM3)
            for (int k = 0; k < 3; ++k) Pn[k] = P.normal[3 * ip + k];
        if (variant == ORBGPU_PROJ_LAST_FRAME) lv = P.octave[ip];
    }
    Query q{};
    if (C.check_ori && (variant == ORBGPU_PROJ_LAST_FRAME || variant == ORBGPU_PROJ_KEYFRAME)) q.angle = P.angle[ip];
    q.level_lo = -1000;
    q.level_hi = 1000;
    q.flags = fl;
    q.ok = (fl & ORBGPU_PT_VALID) != 0;
    if (variant == ORBGPU_PROJ_LOCAL) {  // ORBmatcher.cpp:68-91
        q.ok = q.ok && (fl & ORBGPU_PT_IN_VIEW);
        if (q.ok) {
            float r = (double)tr[3] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos: double literal
            if (C.th != 1.0f) r *= C.th;
            q.u = tr[0];
            q.v = tr[1];
            q.r = r * sf[lv & 15];  // track level validated on the host (0..n_levels-1)
            q.min_level = lv - 1;
            q.max_level = lv;
            q.stereo = true;
            q.ur = tr[2];
            q.stereo_r = q.r;
            q.level_lo = -1000;
            q.level_hi = 1000;
        }
    } else if (variant == ORBGPU_PROJ_SIM3 || variant == ORBGPU_PROJ_FUSE || variant == ORBGPU_PROJ_FUSE_SIM3) {
        // SIM3: ORBmatcher.cpp:376-420; FUSE: :987-1030 (Rcw, tcw of the keyframe,
        // then the same tests); FUSE_SIM3: :1149-1198 (the scale removed as in SIM3)
        if (q.ok) {
            float pc[3];
            transform(variant == ORBGPU_PROJ_FUSE ? T.Tcw : cp.Rs, X, pc);
            if (pc[2] < 0.0f) q.ok = false;
            else {
                const float invz = 1 / pc[2];
                const float x = pc[0] * invz, y = pc[1] * invz;
                q.u = T.fx * x + T.cx;
                q.v = T.fy * y + T.cy;
                if (!(q.u >= T.min_x && q.u < T.max_x && q.v >= T.min_y && q.v < T.max_y)) q.ok = false;  // IsInImage
                q.ur = q.u - T.bf * invz;  // FUSE (:1008)
            }
            if (q.ok) {
                const float maxd = 1.2f * maxd0, mind = 0.8f * mind0;
                const float PO[3] = {X[0] - cp.O[0], X[1] - cp.O[1], X[2] - cp.O[2]};
                const float dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
                if (dist < mind || dist > maxd) q.ok = false;
                else {
                    const double dot = (double)PO[0] * Pn[0] + (double)PO[1] * Pn[1] + (double)PO[2] * Pn[2];
                    if (dot < 0.5 * dist) q.ok = false;
                    else {
                        const int lvl = predict_scale(maxd0, dist, T);
                        q.r = C.th * sf[lvl];
                        q.min_level = -1;
                        q.max_level = -1;
                        q.stereo = false;
                        q.chi2 = variant == ORBGPU_PROJ_FUSE;
                        q.level_lo = lvl - 1;
                        q.level_hi = lvl;
                    }
                }
            }
        }
    } else if (variant == ORBGPU_PROJ_SIM3_DIR) {  // SearchBySim3, one direction (ORBmatcher.cpp:1305-1387)
        if (q.ok) {
            float pc1[3], pc[3];
            transform(C.last_Tcw, X, pc1);  // the points' own keyframe: R1w*p3Dw + t1w
            transform(T.Tcw, pc1, pc);      // the similarity: sR21*p3Dc1 + t21
            if (pc[2] < 0.0f) q.ok = false;
            else {
                const float invz = 1 / pc[2];
                const float x = pc[0] * invz, y = pc[1] * invz;
                q.u = T.fx * x + T.cx;
                q.v = T.fy * y + T.cy;
                if (!(q.u >= T.min_x && q.u < T.max_x && q.v >= T.min_y && q.v < T.max_y)) q.ok = false;
            }
            if (q.ok) {
                const float maxd = 1.2f * maxd0, mind = 0.8f * mind0;
                const float dist = (float)sqrt((double)pc[0] * pc[0] + (double)pc[1] * pc[1] + (double)pc[2] * pc[2]);
                if (dist < mind || dist > maxd) q.ok = false;
                else {
                    const int lvl = predict_scale(maxd0, dist, T);
                    q.r = C.th * sf[lvl];
                    q.min_level = -1;
                    q.max_level = -1;
                    q.level_lo = lvl - 1;
                    q.level_hi = lvl;
                }
            }
        }
    } else {  // LAST_FRAME (ORBmatcher.cpp:1536-1571), KEYFRAME (:1683-1713)
        if (q.ok) {
            float pc[3];
            transform(T.Tcw, X, pc);
            const float invzc = (float)(1.0 / (double)pc[2]);
            if (variant == ORBGPU_PROJ_LAST_FRAME && invzc < 0) q.ok = false;
            q.u = T.fx * pc[0] * invzc + T.cx;
            q.v = T.fy * pc[1] * invzc + T.cy;
            if (q.u < T.min_x || q.u > T.max_x || q.v < T.min_y || q.v > T.max_y) q.ok = false;
            if (q.ok && variant == ORBGPU_PROJ_LAST_FRAME) {
                const int o = lv;  // source octave validated on the host (0..n_levels-1)
                q.r = C.th * sf[o & 15];
                if (cp.forward) { q.min_level = o; q.max_level = -1; }
                else if (cp.backward) { q.min_level = 0; q.max_level = o; }
                else { q.min_level = o - 1; q.max_level = o + 1; }
                q.stereo = true;
                q.ur = q.u - T.bf * invzc;
                q.stereo_r = q.r;
                q.level_lo = -1000;
                q.level_hi = 1000;
            } else if (q.ok) {
                const float PO[3] = {X[0] - cp.O[0], X[1] - cp.O[1], X[2] - cp.O[2]};
                const float dist3D = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
                const float maxd = 1.2f * maxd0, mind = 0.8f * mind0;
                if (dist3D < mind || dist3D > maxd) q.ok = false;
                else {
                    const int lvl = predict_scale(maxd0, dist3D, T);
                    q.r = C.th * sf[lvl];
                    q.min_level = lvl - 1;
                    q.max_level = lvl + 1;
                    q.stereo = false;
                    q.level_lo = -1000;
                    q.level_hi = 1000;
                }
            }
        }
    }
    return q;
}

// a candidate slot is hidden by its occupancy: mvpMapPoints[idx] with
// Observations() > 0 (LOCAL, LAST_FRAME), any MapPoint (KEYFRAME) or
// vpMatched[idx] (SIM3)
// (occupancy is 0, 1 or 2: hidden <=> occ >= hidden_min(variant))
__device__ inline int hidden_min(int variant) {
    return (variant == ORBGPU_PROJ_LOCAL || variant == ORBGPU_PROJ_LAST_FRAME) ? 2 : 1;
}

// The target's feature grid in LDS: the first sorted position of every
// cell, the fields a window test reads stored by sorted position, the hidden
// set, and -- for targets of up to kDescLds keypoints -- the descriptors, so a
// window scan does not touch HBM at all.
struct Grid {
    const float4* kp;                 // by sorted position: x, y, u_right (-1 without stereo), slot | octave << 16
    const unsigned short* cell_start;
    const unsigned* hidw;             // hidden-slot bitmap: slot i is bit i & 31 of word i >> 5
    const uint4* desc;                // by slot, 2 x 16 bytes (LDS copy or the target's HBM array)
    const float* isig;                // mvInvLevelSigma2 by octave (FUSE's chi-square test)
};

__device__ inline int kp_slot(const float4& k) { return (int)(__float_as_uint(k.w) & 0xFFFu); }
// octave clamped to int16: exact for every test made on it (the levels it is
// compared with lie in -2..17, and LOCAL's level equality is between
// candidates that passed the level window)
__device__ inline int kp_octave(const float4& k) { return (int)(short)(__float_as_uint(k.w) >> 16); }

// Candidate keys: Hamming distance << 12 | sorted position.  The reference
// keeps the first best in its candidate order (GetFeaturesInArea's), i.e. the
// smallest key.
constexpr unsigned kNoKey = 0xFFFFFFFFu;
__device__ inline int key_dist(unsigned k) { return (int)(k >> 12); }
__device__ inline int key_pos(unsigned k) { return (int)(k & 0xFFFu); }

// GetFeaturesInArea (Frame.cpp:379-432) with the variant's candidate
// filters: G lanes (sub-lane sl) share the window's candidates, flattened
// over its column runs (candidate f to lane f % G), and call visit(key) for
// every candidate that passes.
template <int G, class Visit>
__device__ __forceinline__ void scan_candidates(const orbgpu_proj_call& C, const Query& q, int ip, const Grid& g, float invW,
                                       float invH, int sl, Visit&& visit) {
    const orbgpu_proj_target& T = C.target;
    const int cx0 = max(0, (int)floorf((q.u - T.min_x - q.r) * invW));
    const int cx1 = min(kGC - 1, (int)ceilf((q.u - T.min_x + q.r) * invW));
    const int cy0 = max(0, (int)floorf((q.v - T.min_y - q.r) * invH));
    const int cy1 = min(kGR - 1, (int)ceilf((q.v - T.min_y + q.r) * invH));
    if (cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0 || cx0 > cx1) return;
    const bool check_levels = q.min_level > 0 || q.max_level >= 0;
    const uint4* dp = reinterpret_cast<const uint4*>(C.points.desc + 32 * (size_t)ip);
    const uint4 pa = dp[0], pb = dp[1];
    int col = cx0;
    int ce = g.cell_start[col * kGR + cy1 + 1];
    int p = g.cell_start[col * kGR + cy0] + sl;
    while (true) {
        while (p >= ce && col < cx1) {  // carry into the next column run
            const int over = p - ce;
            ++col;
            ce = g.cell_start[col * kGR + cy1 + 1];
            p = g.cell_start[col * kGR + cy0] + over;
        }
        if (p >= ce) break;
        const int cur = p;
        p += G;
        const float4 k = g.kp[cur];
        const int oct = kp_octave(k), idx = kp_slot(k);
        if (check_levels) {
            if (oct < q.min_level) continue;
            if (q.max_level >= 0 && oct > q.max_level) continue;
        }
        if (!(fabsf(k.x - q.u) < q.r && fabsf(k.y - q.v) < q.r)) continue;
        if ((g.hidw[idx >> 5] >> (idx & 31)) & 1u) continue;
        if (oct < q.level_lo || oct > q.level_hi) continue;
        if (q.stereo && k.z > 0) {
            const float er = fabsf(q.ur - k.z);
            if (er > q.stereo_r) continue;
        }
        if (q.chi2) {  // Fuse: e2 * mvInvLevelSigma2[kpLevel] against 7.8 (stereo) / 5.99 (double literals)
            const float ex = q.u - k.x, ey = q.v - k.y;
            float e2 = ex * ex + ey * ey;
            double lim = 5.99;
            if (k.z >= 0.0f) {
                const float er = q.ur - k.z;
                e2 = e2 + er * er;
                lim = 7.8;
            }
            if ((double)(e2 * g.isig[oct & 15]) > lim) continue;
        }
        const uint4 ea = g.desc[2 * idx], eb = g.desc[2 * idx + 1];
        const int dist = __popc(pa.x ^ ea.x) + __popc(pa.y ^ ea.y) + __popc(pa.z ^ ea.z) + __popc(pa.w ^ ea.w) +
                         __popc(pb.x ^ eb.x) + __popc(pb.y ^ eb.y) + __popc(pb.z ^ eb.z) + __popc(pb.w ^ eb.w);
        visit(((unsigned)dist << 12) | (unsigned)cur);
    }
}

// minimum over aligned groups of G lanes
template <int G>
__device__ inline unsigned gmin32(unsigned v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    return v;
}

// best / second best (smallest keys) over the wave, current hidden set
__device__ inline void best_two(const orbgpu_proj_call& C, const Query& q, int ip, const Grid& g, float invW,
                                float invH, int lane, unsigned& b1, unsigned& b2) {
    unsigned best = kNoKey, best2 = kNoKey;
    scan_candidates<64>(C, q, ip, g, invW, invH, lane, [&](unsigned key) {
        best2 = key < best ? best : min(key, best2);
        best = min(key, best);
    });
    b1 = gmin32<64>(best);
    b2 = gmin32<64>(best == b1 ? best2 : best);
}

// rotation bin of a match (ORBmatcher.cpp:155-163 and the overloads' copies)
__device__ inline int rot_bin(float src_angle, float kp_angle) {
    float rot = src_angle - kp_angle;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * ((float)kHL / 360.0f));
    if (bin == kHL) bin = 0;
    return bin;
}

#ifdef PROJ_STAMPS  // diagnostic: per-phase wall-clock of each call, printed by thread 0
#define PSTAMP(k) do { if (tid == 0 && (k) < 16) st_[k] = wall_clock64(); } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif

constexpr int kProjThreads = 1024;       // 16 waves: 15 build candidate lists, 1 resolves
constexpr int kListK = 4;                // candidates kept per point (smallest keys)
constexpr int kSub = 4;                  // lanes per point while building lists (one list entry each)
constexpr int kChunk = 240;              // points per list buffer (one round of the 15 list waves)
constexpr int kDescLds = 2048;           // targets up to this size keep their descriptors in LDS
// dynamic LDS: per keypoint kp (16 B) | angle (4) | first hider (4) | rotHist bins (4) [| descriptor (32)]
constexpr int kProjDynLds = 28 * kMaxKps > 60 * kDescLds ? 28 * kMaxKps : 60 * kDescLds;

// list entry aux word: slot | rotation bin << 12 | (int8) octave << 17
__device__ inline int aux_slot(unsigned a) { return (int)(a & 0xFFFu); }
__device__ inline int aux_bin(unsigned a) { return (int)((a >> 12) & 31u); }
__device__ inline int aux_octave(unsigned a) { return (int)(signed char)(a >> 17); }

// One block per call.  Phase 1 (all threads): the target's 64x48 feature
// grid in LDS (AssignFeaturesToGrid, Frame.cpp:241-259): (cell, slot) keys
// placed by a counting sort over the cells with insertion order restored
// within each cell, so a cell row ix, cells iy0..iy1, is one contiguous run
// in GetFeaturesInArea's order (ix outer, iy inner, insertion order); the
// hidden-slot bitmap; the descriptors when they fit.  Phase 2: the
// reference walks the points in order and an assignment hides a keypoint
// from later points, so:
//   * waves 1..15, kSub lanes per point, project every point of the next
//     chunk and keep its kListK smallest candidate keys with the candidates'
//     slot, octave and rotation bin, and its candidate count -- the hidden
//     set only grows as the walk goes on, so a list built early holds the
//     later truth's best candidates in order;
//   * wave 0 replays the walk over the current chunk 64 points at a time
//     (lane = point): every lane resolves its point from its list against
//     the hidden set, then the lanes up to the first one whose examined
//     entries hold a slot an earlier lane of the batch hides (or whose
//     truncated list ran out) commit together; that lane is re-resolved
//     (or rescanned exactly) and the batch goes on from it.  The result is
//     the sequential walk's: a committed lane saw exactly the hidden set the
//     reference's loop sees at its point.
// The two list buffers alternate, so building chunk c+1 overlaps resolving
// chunk c.  Matches are written with atomic max over the point index (the
// reference's last assignment of a slot wins).  Phase 3 applies the
// rotation-consistency cull (LAST_FRAME, KEYFRAME).
__global__ __launch_bounds__(kProjThreads) void proj_kernel(const orbgpu_proj_call* __restrict__ calls, int stride,
                                                            int* __restrict__ match_g, int* __restrict__ nmatches) {
    __shared__ unsigned short s_cell_start[kCells + 1];
    __shared__ unsigned int s_hidw[kMaxKps / 32];  // hidden slots (occupancy >= hidden_min)
    __shared__ uint2 s_list[2][kChunk][kListK];    // (key, aux) per list entry
    __shared__ int s_ncand[2][kChunk];             // candidate count | has-observations << 30; -1: no query
    __shared__ int s_hist[kHL];
    __shared__ float s_sf[16], s_isig[16];
    __shared__ int s_nm;  // per-point variants: accepted points
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const orbgpu_proj_call& C = calls[blockIdx.x];
    const orbgpu_proj_target& T = C.target;
    const orbgpu_proj_points& P = C.points;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int* match = match_g + (size_t)blockIdx.x * stride;
#ifdef PROJ_STAMPS
    unsigned long long st_[16] = {};
#endif
    PSTAMP(0);
    const int n = T.n;
    const int variant = C.variant, np = P.n;
    const bool perpoint = per_point(variant);
    // the output row holds one entry per target keypoint (per point for the per-point variants)
    if (n > kMaxKps || (perpoint ? np : n) > stride) {
        if (tid == 0) nmatches[blockIdx.x] = -1;
        return;
    }
    const int hmin = perpoint ? 3 : hidden_min(variant);  // per-point variants hide nothing
    const bool desc_lds = n <= kDescLds;
    const int nr = (n + 3) & ~3;
    float4* s_kp = reinterpret_cast<float4*>(s_dyn);
    float* s_kang = reinterpret_cast<float*>(s_dyn + 16 * nr);
    unsigned* s_first = reinterpret_cast<unsigned*>(s_dyn + 20 * nr);  // walk: lowest batch lane hiding a slot
    unsigned* s_bins = reinterpret_cast<unsigned*>(s_dyn + 24 * nr);   // per slot: rotHist bins holding it
    uint4* s_desc = reinterpret_cast<uint4*>(s_dyn + 28 * nr);
    int* s_cnt = reinterpret_cast<int*>(&s_list[0][0][0]);  // phase 1: per-cell counts, then cursors
    unsigned* s_sorted = s_first;                            // phase 1: (cell << 12 | slot) keys (8n bytes free)
    // ---- phase 1: grid (PosInGrid with C round, Frame.cpp:434-443) by a counting sort over the cells
    const float invW = (float)kGC / (T.max_x - T.min_x), invH = (float)kGR / (T.max_y - T.min_y);
    for (int c = tid; c < kCells; c += kProjThreads) s_cnt[c] = 0;
    if (const uint8_t* occ = perpoint ? nullptr : T.occupied) {  // hidden-slot bitmap, 64 slots per ballot
        for (int i0 = wave * 64; i0 < n; i0 += kProjThreads) {
            const int i = i0 + lane;
            const unsigned long long m = __ballot(i < n && occ[i] >= hmin);
            if (lane == 0) {
                s_hidw[i0 >> 5] = (unsigned)m;
                s_hidw[(i0 >> 5) + 1] = (unsigned)(m >> 32);
            }
        }
    } else {
        for (int w = tid; w < kMaxKps / 32; w += kProjThreads) s_hidw[w] = 0;
    }
    if (tid < kHL) s_hist[tid] = 0;
    if (tid < 16) {
        const float sfl = tid < T.n_levels ? T.scale_factors[tid] : 0.0f;
        s_sf[tid] = sfl;
        s_isig[tid] = 1.0f / (sfl * sfl);  // mvInvLevelSigma2 = 1 / (s * s) (ORBextractor.cpp:428-433)
    }
    if (tid == 0) s_nm = 0;
    if (desc_lds) {  // the descriptors, 16 bytes per piece, four pieces per thread in flight before any store
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // (arrays of HIP's uint4 land in scratch)
        const v4u* gd = reinterpret_cast<const v4u*>(T.desc);
        v4u* sd = reinterpret_cast<v4u*>(s_desc);
        for (int i0 = tid; i0 < 2 * n; i0 += 4 * kProjThreads) {
            v4u v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = gd[min(i0 + k * kProjThreads, 2 * n - 1)];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i0 + k * kProjThreads < 2 * n) sd[i0 + k * kProjThreads] = v[k];
        }
    }
    __syncthreads();
    constexpr int kPer = kMaxKps / kProjThreads;
    int cell[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        const int i = tid + r * kProjThreads;
        cell[r] = -1;
        if (i < n) {
            const int px = (int)roundf((T.kps[i].x - T.min_x) * invW);
            const int py = (int)roundf((T.kps[i].y - T.min_y) * invH);
            if (px >= 0 && px < kGC && py >= 0 && py < kGR) {
                cell[r] = px * kGR + py;
                atomicAdd(&s_cnt[cell[r]], 1);
            }
        }
    }
    __syncthreads();
    {  // exclusive scan of the counts: 3 cells per thread, wave scans, wave totals
        constexpr int kCPT = kCells / kProjThreads;
        int c3[kCPT], loc = 0;
#pragma unroll
        for (int k = 0; k < kCPT; ++k) {
            c3[k] = s_cnt[kCPT * tid + k];
            loc += c3[k];
        }
        const int v = wave_incl_scan_dpp(loc);
        int* s_wsum = s_ncand[0];  // 16 wave totals (s_ncand is free until the lists)
        if (lane == 63) s_wsum[wave] = v;
        __syncthreads();
        int off = v - loc;
        for (int w = 0; w < wave; ++w) off += s_wsum[w];
#pragma unroll
        for (int k = 0; k < kCPT; ++k) {
            s_cell_start[kCPT * tid + k] = (unsigned short)off;
            s_cnt[kCPT * tid + k] = off;
            off += c3[k];
        }
        if (tid == kProjThreads - 1) s_cell_start[kCells] = (unsigned short)off;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer; ++r)  // scatter (any order within a cell)
        if (cell[r] >= 0) s_sorted[atomicAdd(&s_cnt[cell[r]], 1)] = ((unsigned)cell[r] << 12) | (unsigned)(tid + r * kProjThreads);
    __syncthreads();
    for (int c = tid; c < kCells; c += kProjThreads) {  // insertion order within each cell
        const int s0 = s_cell_start[c], e0 = s_cell_start[c + 1];
        for (int x = s0 + 1; x < e0; ++x) {
            const unsigned key = s_sorted[x];
            int y = x - 1;
            while (y >= s0 && s_sorted[y] > key) {
                s_sorted[y + 1] = s_sorted[y];
                --y;
            }
            s_sorted[y + 1] = key;
        }
    }
    __syncthreads();
    const int ngrid = s_cell_start[kCells];
    for (int p = tid; p < ngrid; p += kProjThreads) {  // window-test fields in sorted order
        const int i = (int)(s_sorted[p] & 0xFFFu);
        const orbgpu_keypoint kp = T.kps[i];
        const unsigned oct = (unsigned)(unsigned short)(short)min(32767, max(-32768, kp.octave));
        s_kp[p] = make_float4(kp.x, kp.y, T.u_right ? T.u_right[i] : -1.0f, __uint_as_float((unsigned)i | oct << 16));
        s_kang[p] = kp.angle;
    }
    __syncthreads();
    for (int i = tid; i < n; i += kProjThreads) {  // the sort keys are consumed
        s_first[i] = ~0u;
        s_bins[i] = 0u;
    }
    PSTAMP(1);
    const Grid g{s_kp, s_cell_start, s_hidw, desc_lds ? s_desc : reinterpret_cast<const uint4*>(T.desc), s_isig};
    const int pp_max = variant == ORBGPU_PROJ_SIM3_DIR ? kThHigh : kThLow;  // per-point acceptance
    const CallPose cp = call_pose(C);
    const bool hist = C.check_ori && (variant == ORBGPU_PROJ_LAST_FRAME || variant == ORBGPU_PROJ_KEYFRAME);
    // list of chunk ch into buffer ch & 1, by waves w0..15 (nw waves), kSub lanes per point
    auto build = [&](int ch, int w0, int nw) {
        const int buf = ch & 1;
        const int gid = (wave - w0) * (64 / kSub) + lane / kSub, sl = lane % kSub, ng = nw * (64 / kSub);
        for (int jb = 0; jb < kChunk; jb += ng) {
            if (ch * kChunk + jb >= np) break;
            const int j = jb + gid, ip = ch * kChunk + j;
            const bool act = j < kChunk && ip < np;
            Query q{};
            if (act) q = make_query(C, cp, s_sf, ip);
            unsigned top[kListK];
#pragma unroll
            for (int k = 0; k < kListK; ++k) top[k] = kNoKey;
            int cnt = 0;
            if (q.ok)
                scan_candidates<kSub>(C, q, ip, g, invW, invH, sl, [&](unsigned key) {
                    ++cnt;
#pragma unroll
                    for (int k = kListK - 1; k >= 0; --k) {  // insert into the lane's sorted top-K
                        const unsigned prev = k > 0 ? top[k - 1] : 0u;
                        if (key < top[k]) top[k] = (k > 0 && key < prev) ? prev : key;
                    }
                });
#pragma unroll
            for (int o = kSub / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
            // the group's kListK smallest keys: every lane ranks its own keys against the group's
            // (keys are distinct) and writes those of rank < kListK with slot, octave and bin
            unsigned other[kSub - 1][kListK];
#pragma unroll
            for (int o = 1; o < kSub; ++o)
#pragma unroll
                for (int k = 0; k < kListK; ++k) other[o - 1][k] = (unsigned)__shfl_xor((int)top[k], o, 64);
            if (!act) continue;
#pragma unroll
            for (int k = 0; k < kListK; ++k) {
                if (top[k] == kNoKey) break;
                int rank = k;
#pragma unroll
                for (int o = 0; o < kSub - 1; ++o)
#pragma unroll
                    for (int t = 0; t < kListK; ++t) rank += other[o][t] < top[k] ? 1 : 0;
                if (perpoint) {  // the group minimum = the reference's first best in window order
                    if (rank == 0) {
                        const bool okd = key_dist(top[k]) <= pp_max;
                        match[ip] = okd ? kp_slot(s_kp[key_pos(top[k])]) : -1;
                        if (okd) atomicAdd(&s_nm, 1);
                    }
                } else if (rank < kListK) {
                    const float4 kq = s_kp[key_pos(top[k])];
                    const int oct = max(-128, min(127, kp_octave(kq)));
                    const unsigned bin = hist ? (unsigned)rot_bin(q.angle, s_kang[key_pos(top[k])]) : 0u;
                    s_list[buf][j][rank] = make_uint2(top[k], (unsigned)kp_slot(kq) | bin << 12 | ((unsigned)oct & 0xFFu) << 17);
                }
            }
            if (perpoint) {
                if (sl == 0 && cnt == 0) match[ip] = -1;  // no query or an empty window
            } else if (sl == 0) {
                for (int k = min(cnt, kListK); k < kListK; ++k) s_list[buf][j][k] = make_uint2(kNoKey, 0u);
                s_ncand[buf][j] = q.ok ? cnt | ((q.flags & ORBGPU_PT_HAS_OBS) ? (1 << 30) : 0) : -1;
            }
        }
    };
    __syncthreads();
    const int nchunks = (np + kChunk - 1) / kChunk;
    if (perpoint) {  // Fuse / SearchBySim3: independent points, every wave builds
        for (int ch = 0; ch < nchunks; ++ch) build(ch, 0, kProjThreads / 64);
        __syncthreads();
        if (tid == 0) nmatches[blockIdx.x] = s_nm;
        return;
    }
    if (nchunks > 0) build(0, 0, kProjThreads / 64);
    if (wave == 0)  // matches start NULL; wave 0 owns every later write of match[]
        for (int i = lane; i < n; i += 64) match[i] = -1;
    __syncthreads();
    PSTAMP(2);
    // the variant's acceptance of a best (b1, octave o1) / second best (b2, o2) pair
    const int need = variant == ORBGPU_PROJ_LOCAL ? 2 : 1;
    const float nnratio = C.nnratio;
    const int orb_dist = C.orb_dist;
    auto accept = [&](unsigned b1, unsigned b2, int o1, int o2) {
        const int bestDist = key_dist(b1);
        if (variant == ORBGPU_PROJ_LOCAL) {  // ORBmatcher.cpp:133-151
            const int bestDist2 = b2 == kNoKey ? 256 : key_dist(b2);
            const int bestLevel2 = b2 == kNoKey ? -1 : o2;
            return bestDist <= kThHigh && !(o1 == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2);
        }
        if (variant == ORBGPU_PROJ_SIM3) return bestDist <= kThLow;
        if (variant == ORBGPU_PROJ_LAST_FRAME) return bestDist <= kThHigh;
        return bestDist <= orb_dist;
    };
    int nm = 0;
    for (int ch = 0; ch < nchunks; ++ch) {
        if (wave > 0) {
            if (ch + 1 < nchunks) build(ch + 1, 1, kProjThreads / 64 - 1);
        } else {
            // ---- wave 0: the reference's loop over the chunk's points, 64 per batch
            const int buf = ch & 1;
            for (int b = 0; b < kChunk; b += 64) {
                const int ipb = ch * kChunk + b;
                if (ipb >= np) break;
                const int jn = min(64, min(kChunk - b, np - ipb));
                const int ip = ipb + lane;
                int nc = -1;
                uint2 e[kListK];
#pragma unroll
                for (int k = 0; k < kListK; ++k) e[k] = make_uint2(kNoKey, 0u);
                if (lane < jn) {
                    nc = s_ncand[buf][b + lane];
#pragma unroll
                    for (int k = 0; k < kListK; ++k) e[k] = s_list[buf][b + lane][k];
                }
                const bool live = nc > 0;  // a valid point with a non-empty window
                const bool trunc = (nc & ((1 << 30) - 1)) > kListK;
                const bool hides_on_match = ((nc >> 30) & 1 ? 2 : 1) >= hmin;
                int t = 0;  // lanes below t are committed
                while (t < jn) {
                    // every pending lane resolves its point against the current hidden set
                    unsigned b1 = kNoKey, b2 = kNoKey, x1 = 0, x2 = 0, exam[kListK];
                    int nvis = 0;
#pragma unroll
                    for (int k = 0; k < kListK; ++k) {
                        const bool examined = e[k].x != kNoKey && nvis < need;
                        const unsigned i = (unsigned)aux_slot(e[k].y);
                        exam[k] = examined ? i : 0xFFFFFFFFu;
                        const bool vis = examined && !((s_hidw[i >> 5] >> (i & 31)) & 1u);
                        b2 = vis && nvis == 1 ? e[k].x : b2;
                        x2 = vis && nvis == 1 ? e[k].y : x2;
                        b1 = vis && nvis == 0 ? e[k].x : b1;
                        x1 = vis && nvis == 0 ? e[k].y : x1;
                        nvis += vis ? 1 : 0;
                    }
                    const bool pend = lane >= t && lane < jn;
                    const bool rescan = pend && live && nvis < need && trunc;
                    const bool acc = pend && live && !rescan && b1 != kNoKey &&
                                     accept(b1, b2, aux_octave(x1), aux_octave(x2));
                    const bool hides = acc && hides_on_match;
                    // a lane whose examined entries hold a slot an earlier pending lane hides
                    // (s_first: the lowest hiding lane per slot, reset right after the test)
                    const unsigned slot = (unsigned)aux_slot(x1);
                    if (hides) atomicMin(&s_first[slot], (unsigned)lane);
                    bool conflict = false;
#pragma unroll
                    for (int k = 0; k < kListK; ++k)
                        conflict = conflict || (exam[k] != 0xFFFFFFFFu && s_first[exam[k]] < (unsigned)lane);
                    if (hides) s_first[slot] = ~0u;
                    const unsigned long long stop = __ballot(pend && (conflict || rescan));
                    const int t0 = stop ? __builtin_ctzll(stop) : jn;
                    // commit the pending lanes below t0
                    const bool com = acc && lane < t0;
                    if (com) {
                        if (hides) atomicOr(&s_hidw[slot >> 5], 1u << (slot & 31));
                        atomicMax(&match[slot], ip);
                    }
                    if (hist && com) {  // rotHist[bin].push_back(slot)
                        atomicOr(&s_bins[slot], 1u << aux_bin(x1));
                        atomicAdd(&s_hist[aux_bin(x1)], 1);
                    }
                    nm += __popcll(__ballot(com));
                    t = t0;
                    if (t0 < jn && !((__ballot(conflict) >> t0) & 1ull)) {
                        // lane t0's truncated list ran out: rescan its window exactly
                        const int ipr = ipb + t0;
                        const int ncr = __builtin_amdgcn_readlane(nc, t0);
                        const Query q = make_query(C, cp, s_sf, ipr);
                        unsigned r1, r2;
                        best_two(C, q, ipr, g, invW, invH, lane, r1, r2);
                        if (r1 != kNoKey) {
                            const float4 k1 = s_kp[key_pos(r1)];
                            const int q2 = r2 != kNoKey ? kp_octave(s_kp[key_pos(r2)]) : 0;
                            if (accept(r1, r2, kp_octave(k1), q2)) {
                                const unsigned sr = (unsigned)kp_slot(k1);
                                if (lane == 0) {
                                    if (((ncr >> 30) & 1 ? 2 : 1) >= hmin) atomicOr(&s_hidw[sr >> 5], 1u << (sr & 31));
                                    atomicMax(&match[sr], ipr);
                                    if (hist) {
                                        const int bin = rot_bin(q.angle, s_kang[key_pos(r1)]);
                                        atomicOr(&s_bins[sr], 1u << bin);
                                        atomicAdd(&s_hist[bin], 1);
                                    }
                                }
                                ++nm;
                            }
                        }
                        t = t0 + 1;
                    }
                }
            }
            PSTAMP(3 + 2 * ch);
        }
        __syncthreads();
        PSTAMP(4 + 2 * ch);
    }
    // ---- phase 3 (wave 0): rotation-consistency cull
    if (wave != 0) return;
    __threadfence();  // the walk's atomic match updates land before the cull's stores
    if (hist) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;  // ComputeThreeMaxima
        for (int i = 0; i < kHL; ++i) {
            const int s = s_hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) ind3 = -1;
        unsigned keep = 0;
        if (ind1 >= 0) keep |= 1u << ind1;
        if (ind2 >= 0) keep |= 1u << ind2;
        if (ind3 >= 0) keep |= 1u << ind3;
        for (int b = 0; b < kHL; ++b)  // every entry of a culled bin is one match less
            if (!((keep >> b) & 1u)) nm -= s_hist[b];
        for (int i = lane; i < n; i += 64)  // and sets its slot to NULL
            if (s_bins[i] & ~keep) match[i] = -2;
    }
    if (lane == 0) nmatches[blockIdx.x] = nm;
#ifdef PROJ_STAMPS
    if (tid == 0)
        printf("PROJ v%d n%d m%d: grid %llu build0 %llu | walk0 %llu chunk0 %llu | walk1 %llu chunk1 %llu (x10ns)\n",
               C.variant, n, P.n, st_[1] - st_[0], st_[2] - st_[1], st_[3] - st_[2], st_[4] - st_[2],
               st_[5] - st_[4], st_[6] - st_[4]);
#endif
}

__global__ __launch_bounds__(256) void frustum_kernel(orbgpu_proj_target T, int n, const float* __restrict__ pos,
                                                      const float* __restrict__ normal,
                                                      const float* __restrict__ min_dist,
                                                      const float* __restrict__ max_dist, float cos_limit,
                                                      int* __restrict__ flags, float* __restrict__ track,
                                                      int* __restrict__ track_level) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int fl = flags[i] & ~ORBGPU_PT_IN_VIEW;  // mbTrackInView = false (Frame.cpp:307)
    const float* X = pos + 3 * i;
    float pc[3], O[3];
    transform(T.Tcw, X, pc);
    camera_center(T.Tcw, O);
    bool ok = !(pc[2] < 0.0f);
    float u = 0.f, v = 0.f, invz = 0.f, viewCos = 0.f, dist = 0.f;
    if (ok) {
        invz = 1.0f / pc[2];
        u = T.fx * pc[0] * invz + T.cx;
        v = T.fy * pc[1] * invz + T.cy;
        if (u < T.min_x || u > T.max_x || v < T.min_y || v > T.max_y) ok = false;
    }
    if (ok) {
        const float maxd = 1.2f * max_dist[i], mind = 0.8f * min_dist[i];
        const float PO[3] = {X[0] - O[0], X[1] - O[1], X[2] - O[2]};
        dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist < mind || dist > maxd) ok = false;
        else {
            const float* Pn = normal + 3 * i;
            viewCos = (float)(((double)PO[0] * Pn[0] + (double)PO[1] * Pn[1] + (double)PO[2] * Pn[2]) / dist);
            if (viewCos < cos_limit) ok = false;
        }
    }
    if (ok) {
        fl |= ORBGPU_PT_IN_VIEW;
        track[4 * i] = u;
        track[4 * i + 1] = v;
        track[4 * i + 2] = u - T.bf * invz;
        track[4 * i + 3] = viewCos;
        track_level[i] = predict_scale(max_dist[i], dist, T);
    }
    flags[i] = fl;
}

}  // namespace

int proj_max_keypoints() { return kMaxKps; }

hipError_t launch_search_by_projection(int ncalls, const orbgpu_proj_call* calls, int stride, int* match,
                                       int* nmatches, hipStream_t stream) {
    if (ncalls <= 0) return hipSuccess;
    // the kernel's LDS limit, once per device (device_state.h)
    static PerDeviceOnce attr_once;
    const hipError_t attr = attr_once.get([](int) {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&proj_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kProjDynLds);
    });
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(proj_kernel, dim3(ncalls), dim3(kProjThreads), kProjDynLds, stream, calls, stride, match,
                       nmatches);
    return hipGetLastError();
}

hipError_t launch_is_in_frustum(const orbgpu_proj_target& T, int n, const float* pos, const float* normal,
                                const float* min_dist, const float* max_dist, float cos_limit, int* flags,
                                float* track, int* track_level, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(frustum_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, T, n, pos, normal, min_dist,
                       max_dist, cos_limit, flags, track, track_level);
    return hipGetLastError();
}

}  // namespace orbgpu
