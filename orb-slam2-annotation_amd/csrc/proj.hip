// proj.hip -- the projection matchers (include/orbgpu_proj.h):
// Frame::isInFrustum and the four ORBmatcher::SearchByProjection overloads.
//
// One 1024-thread block per call (proj_kernel, below): the target's feature
// grid in LDS, every point's projection and candidate list built by 15
// waves in parallel (8 lanes per point), the reference's sequential point
// walk (an assignment hides a keypoint from later points) replayed by one
// wave from those lists, then the rotation-consistency cull.  Candidate keys (Hamming distance <<
// 20 | grid position) reproduce the reference's first-best-in-order choice.
#include "../../include/orbgpu_proj.h"
#include "proj_kernels.h"

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
    float u, v, r;       // window centre and half-size
    int min_level, max_level;
    float ur;            // stereo: projected right coordinate (LOCAL, LAST_FRAME)
    float stereo_r;      // stereo tolerance
    bool stereo;
    int level_lo, level_hi;  // SIM3: keypoint level window applied after the area query
};

// Per-call pose quantities shared by every point of the call.
struct CallPose {
    float O[3];
    float Rs[16];  // SIM3: [Rcw | tcw] after removing the scale
    bool forward, backward;
};

__device__ inline CallPose call_pose(const orbgpu_proj_call& C) {
    CallPose cp{};
    const orbgpu_proj_target& T = C.target;
    const float* Tcw = T.Tcw;
    if (C.variant == ORBGPU_PROJ_SIM3) {  // ORBmatcher.cpp:361-371
        const float row0[3] = {Tcw[0], Tcw[1], Tcw[2]};
        const float scw = (float)sqrt((double)row0[0] * row0[0] + (double)row0[1] * row0[1] + (double)row0[2] * row0[2]);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) cp.Rs[4 * i + j] = Tcw[4 * i + j] / scw;
            cp.Rs[4 * i + 3] = Tcw[4 * i + 3] / scw;
        }
        camera_center(cp.Rs, cp.O);
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
__device__ inline Query make_query(const orbgpu_proj_call& C, const CallPose& cp, int ip) {
    const orbgpu_proj_target& T = C.target;
    const orbgpu_proj_points& P = C.points;
    const int fl = P.flags[ip];
    Query q{};
    q.ok = (fl & ORBGPU_PT_VALID) != 0;
    if (C.variant == ORBGPU_PROJ_LOCAL) {  // ORBmatcher.cpp:68-91
        q.ok = q.ok && (fl & ORBGPU_PT_IN_VIEW);
        if (q.ok) {
            const int lvl = P.track_level[ip];
            float r = (double)P.track[4 * ip + 3] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos: double literal
            if (C.th != 1.0f) r *= C.th;
            q.u = P.track[4 * ip];
            q.v = P.track[4 * ip + 1];
            q.r = r * T.scale_factors[lvl];
            q.min_level = lvl - 1;
            q.max_level = lvl;
            q.stereo = true;
            q.ur = P.track[4 * ip + 2];
            q.stereo_r = q.r;
            q.level_lo = -1000;
            q.level_hi = 1000;
        }
    } else if (C.variant == ORBGPU_PROJ_SIM3) {  // ORBmatcher.cpp:376-420
        if (q.ok) {
            const float* X = P.pos + 3 * ip;
            float pc[3];
            transform(cp.Rs, X, pc);
            if (pc[2] < 0.0f) q.ok = false;
            else {
                const float invz = 1 / pc[2];
                const float x = pc[0] * invz, y = pc[1] * invz;
                q.u = T.fx * x + T.cx;
                q.v = T.fy * y + T.cy;
                if (!(q.u >= T.min_x && q.u < T.max_x && q.v >= T.min_y && q.v < T.max_y)) q.ok = false;  // IsInImage
            }
            if (q.ok) {
                const float maxd = 1.2f * P.max_dist[ip], mind = 0.8f * P.min_dist[ip];
                const float PO[3] = {X[0] - cp.O[0], X[1] - cp.O[1], X[2] - cp.O[2]};
                const float dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
                if (dist < mind || dist > maxd) q.ok = false;
                else {
                    const float* Pn = P.normal + 3 * ip;
                    const double dot = (double)PO[0] * Pn[0] + (double)PO[1] * Pn[1] + (double)PO[2] * Pn[2];
                    if (dot < 0.5 * dist) q.ok = false;
                    else {
                        const int lvl = predict_scale(P.max_dist[ip], dist, T);
                        q.r = C.th * T.scale_factors[lvl];
                        q.min_level = -1;
                        q.max_level = -1;
                        q.stereo = false;
                        q.level_lo = lvl - 1;
                        q.level_hi = lvl;
                    }
                }
            }
        }
    } else {  // LAST_FRAME (ORBmatcher.cpp:1536-1571), KEYFRAME (:1683-1713)
        if (q.ok) {
            const float* X = P.pos + 3 * ip;
            float pc[3];
            transform(T.Tcw, X, pc);
            const float invzc = (float)(1.0 / (double)pc[2]);
            if (C.variant == ORBGPU_PROJ_LAST_FRAME && invzc < 0) q.ok = false;
            q.u = T.fx * pc[0] * invzc + T.cx;
            q.v = T.fy * pc[1] * invzc + T.cy;
            if (q.u < T.min_x || q.u > T.max_x || q.v < T.min_y || q.v > T.max_y) q.ok = false;
            if (q.ok && C.variant == ORBGPU_PROJ_LAST_FRAME) {
                const int o = P.octave[ip];
                q.r = C.th * T.scale_factors[o];
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
                const float maxd = 1.2f * P.max_dist[ip], mind = 0.8f * P.min_dist[ip];
                if (dist3D < mind || dist3D > maxd) q.ok = false;
                else {
                    const int lvl = predict_scale(P.max_dist[ip], dist3D, T);
                    q.r = C.th * T.scale_factors[lvl];
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

// The target's feature grid in LDS: keypoint slots sorted by cell, the first
// sorted position of every cell, and the fields a window test reads, stored
// in sorted order so a scan touches HBM only for the 32-byte descriptors.
struct Grid {
    const unsigned* sorted;           // cell << 12 | slot
    const unsigned short* cell_start;
    const unsigned* hidw;             // hidden-slot bitmap: slot i is bit i & 31 of word i >> 5
    const float* kx;                  // by sorted position
    const float* ky;
    const int* koct;
    const float* kur;                 // u_right, -1 without stereo
};

// GetFeaturesInArea (Frame.cpp:379-432) with the variant's candidate
// filters; G lanes (sub-lane sl) walk the window's candidates in grid order
// and call visit(key, position) for every candidate that passes, with key =
// Hamming distance << 20 | sorted position: the reference keeps the first
// best in its candidate order, i.e. the smallest key.
template <int G, class Visit>
__device__ inline void scan_candidates(const orbgpu_proj_call& C, const Query& q, int ip, const Grid& g, float invW,
                                       float invH, int sl, Visit&& visit) {
    const orbgpu_proj_target& T = C.target;
    const int cx0 = max(0, (int)floorf((q.u - T.min_x - q.r) * invW));
    const int cx1 = min(kGC - 1, (int)ceilf((q.u - T.min_x + q.r) * invW));
    const int cy0 = max(0, (int)floorf((q.v - T.min_y - q.r) * invH));
    const int cy1 = min(kGR - 1, (int)ceilf((q.v - T.min_y + q.r) * invH));
    if (cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0) return;
    const bool check_levels = q.min_level > 0 || q.max_level >= 0;
    const unsigned long long* dp = reinterpret_cast<const unsigned long long*>(C.points.desc + 32 * (size_t)ip);
    const unsigned long long d0 = dp[0], d1 = dp[1], d2 = dp[2], d3 = dp[3];
    for (int ix = cx0; ix <= cx1; ++ix) {
        const int s = g.cell_start[ix * kGR + cy0], e = g.cell_start[ix * kGR + cy1 + 1];
        for (int p = s + sl; p < e; p += G) {
            const int oct = g.koct[p];
            if (check_levels) {
                if (oct < q.min_level) continue;
                if (q.max_level >= 0 && oct > q.max_level) continue;
            }
            if (!(fabsf(g.kx[p] - q.u) < q.r && fabsf(g.ky[p] - q.v) < q.r)) continue;
            const int idx = (int)(g.sorted[p] & 0xFFFu);
            if ((g.hidw[idx >> 5] >> (idx & 31)) & 1u) continue;
            if (C.variant == ORBGPU_PROJ_SIM3 && (oct < q.level_lo || oct > q.level_hi)) continue;
            const float ur = g.kur[p];
            if (q.stereo && ur > 0) {
                const float er = fabsf(q.ur - ur);
                if (er > q.stereo_r) continue;
            }
            const unsigned long long* e8 = reinterpret_cast<const unsigned long long*>(T.desc + 32 * (size_t)idx);
            const int dist = __popcll(d0 ^ e8[0]) + __popcll(d1 ^ e8[1]) + __popcll(d2 ^ e8[2]) + __popcll(d3 ^ e8[3]);
            visit(((unsigned long long)dist << 20) | (unsigned)p);
        }
    }
}

// minimum over aligned groups of G lanes
template <int G>
__device__ inline unsigned long long gmin64(unsigned long long v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(v, o, 64);
        v = t < v ? t : v;
    }
    return v;
}

// best / second best (smallest keys) over the wave, current occupancy
__device__ inline void best_two(const orbgpu_proj_call& C, const Query& q, int ip, const Grid& g, float invW,
                                float invH, int lane, unsigned long long& b1, unsigned long long& b2) {
    unsigned long long best = ~0ull, best2 = ~0ull;
    scan_candidates<64>(C, q, ip, g, invW, invH, lane, [&](unsigned long long key) {
        const bool first = key < best;  // value selects (a branchy update made the compiler spill the pair)
        best2 = first ? best : (key < best2 ? key : best2);
        best = first ? key : best;
    });
    b1 = gmin64<64>(best);
    b2 = gmin64<64>(best == b1 ? best2 : best);
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
constexpr int kSub = 8;                  // lanes per point while building lists
constexpr int kChunk = 240;              // points per list buffer (2 rounds of the 15 list waves)

// One block per call.  Phase 1 (all threads): the target's 64x48 feature
// grid in LDS (AssignFeaturesToGrid, Frame.cpp:241-259) as (cell, slot)
// keys sorted by a block bitonic sort, so a cell row ix, cells iy0..iy1, is
// one contiguous run in GetFeaturesInArea's order (ix outer, iy inner,
// insertion order), and the hidden-slot bitmap.  Phase 2: the reference
// walks the points in order and an assignment hides a keypoint from later
// points, so:
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
    __shared__ unsigned int s_sorted[kMaxKps];     // (cell << 12 | slot)
    __shared__ unsigned short s_cell_start[kCells + 1];
    __shared__ unsigned int s_hidw[kMaxKps / 32];  // hidden slots (occupancy >= hidden_min)
    __shared__ float s_kx[kMaxKps], s_ky[kMaxKps], s_kur[kMaxKps];
    __shared__ int s_koct[kMaxKps];
    __shared__ unsigned int s_acc[kMaxKps];        // rotHist entries in push order: slot | bin << 16
    __shared__ unsigned long long s_list[2][kChunk][kListK];
    __shared__ unsigned int s_aux[2][kChunk][kListK];  // candidate slot | rotation bin << 12
    __shared__ int s_loct[2][kChunk][kListK];      // candidate octave
    __shared__ int s_ncand[2][kChunk];             // candidate count | has-observations << 30; -1: no query
    __shared__ int s_hist[kHL];
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
    if (n > stride || n > kMaxKps) {
        if (tid == 0) nmatches[blockIdx.x] = -1;
        return;
    }
    const int variant = C.variant, hmin = hidden_min(variant), np = P.n;
    // ---- phase 1: grid (PosInGrid with C round, Frame.cpp:434-443)
    const float invW = (float)kGC / (T.max_x - T.min_x), invH = (float)kGR / (T.max_y - T.min_y);
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = tid; i < n2; i += kProjThreads) {
        unsigned key = 0xFFFFFFFFu;
        if (i < n) {
            const int px = (int)roundf((T.kps[i].x - T.min_x) * invW);
            const int py = (int)roundf((T.kps[i].y - T.min_y) * invH);
            if (px >= 0 && px < kGC && py >= 0 && py < kGR) key = ((unsigned)(px * kGR + py) << 12) | (unsigned)i;
        }
        s_sorted[i] = key;
    }
    if (tid < kMaxKps / 32) {
        unsigned w = 0;
        if (T.occupied)
            for (int b = 0; b < 32; ++b) {
                const int i = 32 * tid + b;
                if (i < n && T.occupied[i] >= hmin) w |= 1u << b;
            }
        s_hidw[tid] = w;
    }
    if (tid < kHL) s_hist[tid] = 0;
    for (int size = 2; size <= n2; size <<= 1)  // bitonic sort
        for (int st = size >> 1; st > 0; st >>= 1) {
            __syncthreads();
            for (int i = tid; i < n2 / 2; i += kProjThreads) {
                const int lo = 2 * i - (i & (st - 1)), hi = lo + st;
                const bool up = (lo & size) == 0;
                const unsigned a = s_sorted[lo], b = s_sorted[hi];
                if ((a > b) == up) {
                    s_sorted[lo] = b;
                    s_sorted[hi] = a;
                }
            }
        }
    __syncthreads();
    for (int c = tid; c <= kCells; c += kProjThreads) {  // first sorted position with cell >= c
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((s_sorted[mid] >> 12) < (unsigned)c) lo = mid + 1; else hi = mid;
        }
        s_cell_start[c] = (unsigned short)lo;
    }
    for (int p = tid; p < n; p += kProjThreads) {  // window-test fields in sorted order
        const unsigned key = s_sorted[p];
        if (key == 0xFFFFFFFFu) continue;  // outside the grid: never scanned
        const int i = (int)(key & 0xFFFu);
        const orbgpu_keypoint kp = T.kps[i];
        s_kx[p] = kp.x;
        s_ky[p] = kp.y;
        s_koct[p] = kp.octave;
        s_kur[p] = T.u_right ? T.u_right[i] : -1.0f;
    }
    PSTAMP(1);
    const Grid g{s_sorted, s_cell_start, s_hidw, s_kx, s_ky, s_koct, s_kur};
    const CallPose cp = call_pose(C);
    const bool hist = C.check_ori && (variant == ORBGPU_PROJ_LAST_FRAME || variant == ORBGPU_PROJ_KEYFRAME);
    // list of chunk ch into buffer ch & 1, by waves w0..15 (nw waves), kSub lanes per point
    auto build = [&](int ch, int w0, int nw) {
        const int buf = ch & 1;
        const int gid = (wave - w0) * (64 / kSub) + lane / kSub, sl = lane % kSub, ng = nw * (64 / kSub);
        for (int jb = 0; jb < kChunk; jb += ng) {
            if (ch * kChunk + jb >= np) break;
            const int j = jb + gid, ip = ch * kChunk + j;
            Query q{};
            if (j < kChunk && ip < np) q = make_query(C, cp, ip);
            unsigned long long top[kListK];
#pragma unroll
            for (int k = 0; k < kListK; ++k) top[k] = ~0ull;
            int cnt = 0;
            if (q.ok)
                scan_candidates<kSub>(C, q, ip, g, invW, invH, sl, [&](unsigned long long key) {
                    ++cnt;
#pragma unroll
                    for (int k = kListK - 1; k >= 0; --k) {  // insert into the lane's sorted top-K
                        const unsigned long long prev = k > 0 ? top[k - 1] : 0ull;
                        if (key < top[k]) top[k] = (k > 0 && key < prev) ? prev : key;
                    }
                });
#pragma unroll
            for (int o = kSub / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
            if (!(j < kChunk && ip < np)) continue;
            // the group's kListK smallest keys: repeatedly take the minimum of the lanes' heads;
            // the owner records it with its candidate's slot, octave and rotation bin
            const float pangle = hist ? P.angle[ip] : 0.0f;
#pragma unroll
            for (int k = 0; k < kListK; ++k) {
                const unsigned long long m = gmin64<kSub>(top[0]);
                if (m == ~0ull ? sl == 0 : top[0] == m) {
                    unsigned aux = 0;
                    int oct = 0;
                    if (m != ~0ull) {
                        const int p = (int)(m & 0xFFFFFu), i = (int)(s_sorted[p] & 0xFFFu);
                        aux = (unsigned)i | (hist ? (unsigned)rot_bin(pangle, T.kps[i].angle) << 12 : 0u);
                        oct = s_koct[p];
#pragma unroll
                        for (int t = 0; t + 1 < kListK; ++t) top[t] = top[t + 1];
                        top[kListK - 1] = ~0ull;
                    }
                    s_list[buf][j][k] = m;
                    s_aux[buf][j][k] = aux;
                    s_loct[buf][j][k] = oct;
                }
            }
            if (sl == 0) s_ncand[buf][j] = q.ok ? cnt | ((P.flags[ip] & ORBGPU_PT_HAS_OBS) ? (1 << 30) : 0) : -1;
        }
    };
    __syncthreads();
    const int nchunks = (np + kChunk - 1) / kChunk;
    if (nchunks > 0) build(0, 0, kProjThreads / 64);
    if (wave == 0)  // matches start NULL; wave 0 owns every later write of match[]
        for (int i = lane; i < n; i += 64) match[i] = -1;
    __syncthreads();
    PSTAMP(2);
    // the variant's acceptance of a best (b1, octave o1) / second best (b2, o2) pair
    const int need = variant == ORBGPU_PROJ_LOCAL ? 2 : 1;
    const float nnratio = C.nnratio;
    const int orb_dist = C.orb_dist;
    auto accept = [&](unsigned long long b1, unsigned long long b2, int o1, int o2) {
        const int bestDist = (int)(b1 >> 20);
        if (variant == ORBGPU_PROJ_LOCAL) {  // ORBmatcher.cpp:133-151
            const int bestDist2 = b2 == ~0ull ? 256 : (int)(b2 >> 20);
            const int bestLevel2 = b2 == ~0ull ? -1 : o2;
            return bestDist <= kThHigh && !(o1 == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2);
        }
        if (variant == ORBGPU_PROJ_SIM3) return bestDist <= kThLow;
        if (variant == ORBGPU_PROJ_LAST_FRAME) return bestDist <= kThHigh;
        return bestDist <= orb_dist;
    };
    int nm = 0, nacc = 0;
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
                unsigned long long kk[kListK];
                unsigned ka[kListK] = {};
                int ko[kListK] = {};
#pragma unroll
                for (int k = 0; k < kListK; ++k) kk[k] = ~0ull;
                if (lane < jn) {
                    nc = s_ncand[buf][b + lane];
#pragma unroll
                    for (int k = 0; k < kListK; ++k) {
                        kk[k] = s_list[buf][b + lane][k];
                        ka[k] = s_aux[buf][b + lane][k];
                        ko[k] = s_loct[buf][b + lane][k];
                    }
                }
                const bool live = nc > 0;  // a valid point with a non-empty window
                const bool trunc = (nc & ((1 << 30) - 1)) > kListK;
                const bool hides_on_match = ((nc >> 30) & 1 ? 2 : 1) >= hmin;
                int t = 0;  // lanes below t are committed
                while (t < jn) {
                    // every pending lane resolves its point against the current hidden set
                    unsigned long long b1 = ~0ull, b2 = ~0ull;
                    unsigned x1 = 0, exam[kListK];
                    int o1 = 0, o2 = 0, nvis = 0;
#pragma unroll
                    for (int k = 0; k < kListK; ++k) {
                        const bool examined = kk[k] != ~0ull && nvis < need;
                        const unsigned i = ka[k] & 0xFFFu;
                        exam[k] = examined ? i : 0xFFFFFFFFu;
                        const bool vis = examined && !((s_hidw[i >> 5] >> (i & 31)) & 1u);
                        b2 = vis && nvis == 1 ? kk[k] : b2;
                        o2 = vis && nvis == 1 ? ko[k] : o2;
                        b1 = vis && nvis == 0 ? kk[k] : b1;
                        x1 = vis && nvis == 0 ? ka[k] : x1;
                        o1 = vis && nvis == 0 ? ko[k] : o1;
                        nvis += vis ? 1 : 0;
                    }
                    const bool pend = lane >= t && lane < jn;
                    const bool rescan = pend && live && nvis < need && trunc;
                    const bool acc = pend && live && !rescan && b1 != ~0ull && accept(b1, b2, o1, o2);
                    const bool hides = acc && hides_on_match;
                    // a lane whose examined entries hold a slot an earlier pending lane hides
                    bool conflict = false;
                    unsigned long long hm = __ballot(hides);
                    while (hm) {
                        const int s = __builtin_ctzll(hm);
                        hm &= hm - 1;
                        const unsigned hs = (unsigned)__builtin_amdgcn_readlane((int)(x1 & 0xFFFu), s);
                        bool in = false;
#pragma unroll
                        for (int k = 0; k < kListK; ++k) in = in || exam[k] == hs;
                        conflict = conflict || (lane > s && in);
                    }
                    const unsigned long long stop = __ballot(pend && (conflict || rescan));
                    const int t0 = stop ? __builtin_ctzll(stop) : jn;
                    // commit the pending lanes below t0
                    const bool com = acc && lane < t0;
                    const unsigned slot = x1 & 0xFFFu;
                    if (com) {
                        if (hides) atomicOr(&s_hidw[slot >> 5], 1u << (slot & 31));
                        atomicMax(&match[slot], ip);
                    }
                    const unsigned long long cm = __ballot(com);
                    if (hist) {
                        if (com) {
                            const int r = nacc + __builtin_amdgcn_mbcnt_hi((unsigned)(cm >> 32),
                                                                           __builtin_amdgcn_mbcnt_lo((unsigned)cm, 0u));
                            const unsigned bin = x1 >> 12;
                            if (r < kMaxKps) s_acc[r] = slot | (bin << 16);
                            atomicAdd(&s_hist[bin], 1);
                        }
                        nacc += __popcll(cm);
                    }
                    nm += __popcll(cm);
                    t = t0;
                    if (t0 < jn && !((__ballot(conflict) >> t0) & 1ull)) {
                        // lane t0's truncated list ran out: rescan its window exactly
                        const int ipr = ipb + t0;
                        const int ncr = __builtin_amdgcn_readlane(nc, t0);
                        const Query q = make_query(C, cp, ipr);
                        unsigned long long r1, r2;
                        best_two(C, q, ipr, g, invW, invH, lane, r1, r2);
                        if (r1 != ~0ull) {
                            const int p1 = (int)(r1 & 0xFFFFFu);
                            const int q1 = s_koct[p1], q2 = r2 != ~0ull ? s_koct[r2 & 0xFFFFFu] : 0;
                            if (accept(r1, r2, q1, q2)) {
                                const unsigned sr = s_sorted[p1] & 0xFFFu;
                                if (lane == 0) {
                                    if (((ncr >> 30) & 1 ? 2 : 1) >= hmin) atomicOr(&s_hidw[sr >> 5], 1u << (sr & 31));
                                    atomicMax(&match[sr], ipr);
                                    if (hist) {
                                        const int bin = rot_bin(P.angle[ipr], T.kps[sr].angle);
                                        if (nacc < kMaxKps) s_acc[nacc] = sr | ((unsigned)bin << 16);
                                        atomicAdd(&s_hist[bin], 1);
                                    }
                                }
                                if (hist) ++nacc;
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
        if (nacc > kMaxKps) {  // more histogram entries than the LDS list holds: rejected
            if (lane == 0) nmatches[blockIdx.x] = -1;
            return;
        }
        int culled = 0;
        for (int k = lane; k < nacc; k += 64) {
            const int b = (int)(s_acc[k] >> 16);
            if (b != ind1 && b != ind2 && b != ind3) ++culled;
        }
        for (int k = lane; k < nacc; k += 64) {  // every entry of a culled bin sets its slot to NULL
            const int b = (int)(s_acc[k] >> 16);
            if (b != ind1 && b != ind2 && b != ind3) match[s_acc[k] & 0xFFFFu] = -2;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) culled += __shfl_xor(culled, o, 64);
        nm -= culled;
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
    hipLaunchKernelGGL(proj_kernel, dim3(ncalls), dim3(kProjThreads), 0, stream, calls, stride, match, nmatches);
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
