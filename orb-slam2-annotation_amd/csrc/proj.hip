// proj.hip -- the projection matchers (include/orbgpu_proj.h):
// Frame::isInFrustum and the four ORBmatcher::SearchByProjection overloads.
//
// One 64-lane wave per call.  Phase 1 builds the target's 64x48 feature grid
// in LDS (AssignFeaturesToGrid, Frame.cpp:241-259): (cell, index) keys are
// sorted, so a cell row ix, cells iy0..iy1, is one contiguous run in the
// order GetFeaturesInArea returns (ix outer, iy inner, insertion order).
// Phase 2 walks the points in order -- the reference's loop is sequential
// because an assignment hides a keypoint from later points -- projecting
// each point (variant-specific float arithmetic, cv::Mat products
// accumulated in double) and spreading its candidate keypoints over the
// lanes: window and level filters, occupancy, stereo check, 256-bit Hamming
// distance, then wave min-reductions of (distance, grid order) keys give the
// reference's first best (and second best for LOCAL).  Phase 3 applies the
// rotation-consistency cull (LAST_FRAME, KEYFRAME).
#include "../../include/orbgpu_proj.h"
#include "proj_kernels.h"

namespace orbgpu {

namespace {

constexpr int kMaxKps = 4096;
constexpr int kGC = 64, kGR = 48, kCells = kGC * kGR;
constexpr int kHL = 30, kThLow = 50, kThHigh = 100;

__device__ inline unsigned long long wmin64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(v, o, 64);
        v = t < v ? t : v;
    }
    return v;
}

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

__global__ __launch_bounds__(64) void proj_kernel(const orbgpu_proj_call* __restrict__ calls, int stride,
                                                  int* __restrict__ match_g, int* __restrict__ nmatches) {
    __shared__ unsigned int s_sorted[kMaxKps];     // (cell << 12 | idx), later idx only
    __shared__ unsigned short s_cell_start[kCells + 1];
    __shared__ unsigned char s_occ[kMaxKps];       // occupancy (0 / 1 no obs / 2 with obs)
    __shared__ unsigned int s_acc[kMaxKps];        // rotHist entries in push order: slot | bin << 16
    __shared__ int s_hist[kHL];
    const orbgpu_proj_call& C = calls[blockIdx.x];
    const orbgpu_proj_target& T = C.target;
    const orbgpu_proj_points& P = C.points;
    const int lane = threadIdx.x;
    int* match = match_g + (size_t)blockIdx.x * stride;
    const int n = T.n;
    if (n > stride || n > kMaxKps) {
        if (lane == 0) nmatches[blockIdx.x] = -1;
        return;
    }
    // ---- phase 1: grid (PosInGrid with C round, Frame.cpp:434-443)
    const float invW = (float)kGC / (T.max_x - T.min_x), invH = (float)kGR / (T.max_y - T.min_y);
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = lane; i < n2; i += 64) {
        unsigned key = 0xFFFFFFFFu;
        if (i < n) {
            const int px = (int)roundf((T.kps[i].x - T.min_x) * invW);
            const int py = (int)roundf((T.kps[i].y - T.min_y) * invH);
            if (px >= 0 && px < kGC && py >= 0 && py < kGR) key = ((unsigned)(px * kGR + py) << 12) | (unsigned)i;
        }
        s_sorted[i] = key;
        if (i < n) {
            match[i] = -1;
            s_occ[i] = T.occupied ? T.occupied[i] : 0;
        }
    }
    if (lane < kHL) s_hist[lane] = 0;
    for (int size = 2; size <= n2; size <<= 1)  // bitonic sort, one wave
        for (int st = size >> 1; st > 0; st >>= 1) {
            __syncthreads();
            for (int i = lane; i < n2 / 2; i += 64) {
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
    for (int c = lane; c <= kCells; c += 64) {  // first sorted position with cell >= c
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((s_sorted[mid] >> 12) < (unsigned)c) lo = mid + 1; else hi = mid;
        }
        s_cell_start[c] = (unsigned short)lo;
    }
    __syncthreads();
    // ---- per-call pose
    float O[3], twc[3], tlc_z = 0.f;
    float Rs[16];  // SIM3: [Rcw | tcw] after removing the scale
    const float* Tcw = T.Tcw;
    bool forward = false, backward = false;
    if (C.variant == ORBGPU_PROJ_SIM3) {  // ORBmatcher.cpp:361-371
        const float row0[3] = {Tcw[0], Tcw[1], Tcw[2]};
        const float scw = (float)sqrt((double)row0[0] * row0[0] + (double)row0[1] * row0[1] + (double)row0[2] * row0[2]);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) Rs[4 * i + j] = Tcw[4 * i + j] / scw;
            Rs[4 * i + 3] = Tcw[4 * i + 3] / scw;
        }
        camera_center(Rs, O);
    } else if (C.variant == ORBGPU_PROJ_LAST_FRAME || C.variant == ORBGPU_PROJ_KEYFRAME) {
        camera_center(Tcw, twc);  // twc = -Rcw^T tcw (= Ow)
        for (int j = 0; j < 3; ++j) O[j] = twc[j];
        if (C.variant == ORBGPU_PROJ_LAST_FRAME) {  // ORBmatcher.cpp:1521-1527
            const float* L = C.last_Tcw;
            const float r2[3] = {L[8], L[9], L[10]};
            tlc_z = dotd3(r2, twc) + L[11];
            forward = tlc_z > T.b && !C.mono;
            backward = -tlc_z > T.b && !C.mono;
        }
    }
    const float factor = (float)kHL / 360.0f;
    int nm = 0, nacc = 0;
    // ---- phase 2: points in order
    for (int ip = 0; ip < P.n; ++ip) {
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
                transform(Rs, X, pc);
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
                    const float PO[3] = {X[0] - O[0], X[1] - O[1], X[2] - O[2]};
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
                transform(Tcw, X, pc);
                const float invzc = (float)(1.0 / (double)pc[2]);
                if (C.variant == ORBGPU_PROJ_LAST_FRAME && invzc < 0) q.ok = false;
                q.u = T.fx * pc[0] * invzc + T.cx;
                q.v = T.fy * pc[1] * invzc + T.cy;
                if (q.u < T.min_x || q.u > T.max_x || q.v < T.min_y || q.v > T.max_y) q.ok = false;
                if (q.ok && C.variant == ORBGPU_PROJ_LAST_FRAME) {
                    const int o = P.octave[ip];
                    q.r = C.th * T.scale_factors[o];
                    if (forward) { q.min_level = o; q.max_level = -1; }
                    else if (backward) { q.min_level = 0; q.max_level = o; }
                    else { q.min_level = o - 1; q.max_level = o + 1; }
                    q.stereo = true;
                    q.ur = q.u - T.bf * invzc;
                    q.stereo_r = q.r;
                    q.level_lo = -1000;
                    q.level_hi = 1000;
                } else if (q.ok) {
                    const float PO[3] = {X[0] - O[0], X[1] - O[1], X[2] - O[2]};
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
        if (!q.ok) continue;
        // GetFeaturesInArea (Frame.cpp:379-432) with the variant's candidate filters
        const int cx0 = max(0, (int)floorf((q.u - T.min_x - q.r) * invW));
        const int cx1 = min(kGC - 1, (int)ceilf((q.u - T.min_x + q.r) * invW));
        const int cy0 = max(0, (int)floorf((q.v - T.min_y - q.r) * invH));
        const int cy1 = min(kGR - 1, (int)ceilf((q.v - T.min_y + q.r) * invH));
        if (cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0) continue;
        const bool check_levels = q.min_level > 0 || q.max_level >= 0;
        const uint8_t* dp = P.desc + 32 * (size_t)ip;
        const unsigned long long d0 = reinterpret_cast<const unsigned long long*>(dp)[0],
                                 d1 = reinterpret_cast<const unsigned long long*>(dp)[1],
                                 d2 = reinterpret_cast<const unsigned long long*>(dp)[2],
                                 d3 = reinterpret_cast<const unsigned long long*>(dp)[3];
        unsigned long long best = ~0ull, best2 = ~0ull;  // (dist << 20 | sorted position)
        for (int ix = cx0; ix <= cx1; ++ix) {
            const int s = s_cell_start[ix * kGR + cy0], e = s_cell_start[ix * kGR + cy1 + 1];
            for (int p = s + lane; p < e; p += 64) {
                const int idx = (int)(s_sorted[p] & 0xFFFu);
                const orbgpu_keypoint kp = T.kps[idx];
                if (check_levels) {
                    if (kp.octave < q.min_level) continue;
                    if (q.max_level >= 0 && kp.octave > q.max_level) continue;
                }
                if (!(fabsf(kp.x - q.u) < q.r && fabsf(kp.y - q.v) < q.r)) continue;
                const int occ = s_occ[idx];
                if (C.variant == ORBGPU_PROJ_LOCAL || C.variant == ORBGPU_PROJ_LAST_FRAME) {
                    if (occ == 2) continue;  // mvpMapPoints[idx] with Observations() > 0
                } else if (occ) {
                    continue;  // any MapPoint (KEYFRAME) / vpMatched[idx] (SIM3)
                }
                if (C.variant == ORBGPU_PROJ_SIM3 && (kp.octave < q.level_lo || kp.octave > q.level_hi)) continue;
                if (q.stereo && T.u_right && T.u_right[idx] > 0) {
                    const float er = fabsf(q.ur - T.u_right[idx]);
                    if (er > q.stereo_r) continue;
                }
                const unsigned long long* e8 = reinterpret_cast<const unsigned long long*>(T.desc + 32 * (size_t)idx);
                const int dist = __popcll(d0 ^ e8[0]) + __popcll(d1 ^ e8[1]) + __popcll(d2 ^ e8[2]) + __popcll(d3 ^ e8[3]);
                const unsigned long long key = ((unsigned long long)dist << 20) | (unsigned)p;
                if (key < best) {
                    best2 = best;
                    best = key;
                } else if (key < best2) {
                    best2 = key;
                }
            }
        }
        const unsigned long long wb = wmin64(best);
        if (wb == ~0ull) continue;
        const int bestDist = (int)(wb >> 20);
        const int bestIdx = (int)(s_sorted[wb & 0xFFFFFu] & 0xFFFu);
        bool accept;
        if (C.variant == ORBGPU_PROJ_LOCAL) {  // ORBmatcher.cpp:133-151
            const unsigned long long contrib = best == wb ? best2 : best;
            const unsigned long long w2 = wmin64(contrib);
            const int bestDist2 = w2 == ~0ull ? 256 : (int)(w2 >> 20);
            const int bestLevel = T.kps[bestIdx].octave;
            const int bestLevel2 = w2 == ~0ull ? -1 : T.kps[s_sorted[w2 & 0xFFFFFu] & 0xFFFu].octave;
            accept = bestDist <= kThHigh && !(bestLevel == bestLevel2 && (float)bestDist > C.nnratio * (float)bestDist2);
        } else if (C.variant == ORBGPU_PROJ_SIM3) {
            accept = bestDist <= kThLow;
        } else if (C.variant == ORBGPU_PROJ_LAST_FRAME) {
            accept = bestDist <= kThHigh;
        } else {
            accept = bestDist <= C.orb_dist;
        }
        if (!accept) continue;
        const bool hist = C.check_ori && (C.variant == ORBGPU_PROJ_LAST_FRAME || C.variant == ORBGPU_PROJ_KEYFRAME);
        if (lane == 0) {
            match[bestIdx] = ip;
            s_occ[bestIdx] = (fl & ORBGPU_PT_HAS_OBS) ? 2 : 1;
            if (hist && nacc < kMaxKps) {
                float rot = P.angle[ip] - T.kps[bestIdx].angle;
                if (rot < 0.0f) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == kHL) bin = 0;
                s_acc[nacc] = (unsigned)bestIdx | ((unsigned)bin << 16);
                s_hist[bin] += 1;
            }
        }
        if (hist) ++nacc;
        ++nm;
        __syncthreads();
    }
    __syncthreads();
    // ---- phase 3: rotation-consistency cull
    if (C.check_ori && (C.variant == ORBGPU_PROJ_LAST_FRAME || C.variant == ORBGPU_PROJ_KEYFRAME)) {
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
        __syncthreads();
        for (int k = lane; k < nacc; k += 64) {  // every entry of a culled bin sets its slot to NULL
            const int b = (int)(s_acc[k] >> 16);
            if (b != ind1 && b != ind2 && b != ind3) match[s_acc[k] & 0xFFFFu] = -2;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) culled += __shfl_xor(culled, o, 64);
        nm -= culled;
    }
    if (lane == 0) nmatches[blockIdx.x] = nm;
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
    hipLaunchKernelGGL(proj_kernel, dim3(ncalls), dim3(64), 0, stream, calls, stride, match, nmatches);
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
