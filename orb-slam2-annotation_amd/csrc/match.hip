// match.hip -- ORBmatcher::SearchForInitialization (ORBmatcher.cpp:474-590)
// with Frame::GetFeaturesInArea / AssignFeaturesToGrid semantics
// (Frame.cpp:241-259, :379-443) for distortion-free frames.
//
// One wave per frame pair.  Only octave-0 keypoints take part (F1 queries
// skip level > 0, F2 candidates are filtered to level 0), and in extractor
// output order they are the first n0 keypoints of each frame, so F2's
// level-0 set (positions, 64x48 grid cell, descriptors, matched distance,
// reverse match) lives in LDS.  The query loop is sequential by contract
// (vMatchedDistance and the "steal" of an earlier match feed later queries,
// SURVEY H5); inside a query the candidates are spread over the 64 lanes:
// window/grid test, 256-bit Hamming via 4x popcll, then a wave min-reduction
// of (dist, grid-order key) -- the reference keeps the FIRST minimum in
// GetFeaturesInArea order (cell ix outer, iy inner, index) -- and a second
// reduction for bestDist2.  The rotation histogram, ComputeThreeMaxima and
// the cull run on the same wave.
#include <cstdlib>
#include <type_traits>

#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "../../include/orbgpu.h"
#include "group_sum.h"

namespace orbgpu {

namespace {

// Level-0 keypoints per frame held in LDS.  The 512 variant covers
// nfeatures <= 2350; pairs above it are handed to the 1024 variant (the
// 2x-features initialisation extractor of KITTI mono, Tracking.cpp:149, has
// ~870 at level 0), pairs above that to the 2048 variant (F2's descriptors
// read from HBM instead of LDS: 68 B of LDS per keypoint; initialisation
// extractors up to ~9,400 features); above 2048 a pair reports -1.  A
// variant is launched only when a frame's keypoint capacity can exceed the
// previous one's limit.
constexpr int kMaxK0Small = 512, kMaxK0Large = 1024, kMaxK0Huge = 2048;
constexpr int kMaxK0Tiny = 256;  // launched alone, when the caller bounds level 0 by 256
constexpr int kNeedLarge = -2;  // nmatches sentinel: the pair waits for the large variant
constexpr int kNeedHuge = -3;   // ... for the huge variant
constexpr int kGC = 64, kGR = 48, kHL = 30, kThLow = 50;

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(v, o, 64);
        v = t < v ? t : v;
    }
    return v;
}

__device__ inline int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

constexpr int kBatchThreads = 256;
constexpr int kTopK = 4;  // best candidate keys kept per query by the parallel phase

// (dist, grid order) of a candidate as one ordered key: dist <= 256 (9 bits),
// cell = ix * 48 + iy < 3072 (12 bits), level-0 index < 2048 (11 bits)
constexpr int kKeyJBits = 11;
constexpr uint32_t kKeyJMask = (1u << kKeyJBits) - 1;
__device__ inline uint32_t cand_key(int dist, int cell, int j) {
    return ((uint32_t)dist << (12 + kKeyJBits)) | ((uint32_t)cell << kKeyJBits) | (uint32_t)j;
}
__device__ inline int key_dist(uint32_t key) { return (int)(key >> (12 + kKeyJBits)); }
__device__ inline int key_j(uint32_t key) { return (int)(key & kKeyJMask); }

// Two phases per frame pair (one block of kMatchThreads threads):
//  1 parallel, one thread per F1 query: the F2 level-0 keypoints of the
//    query's window, walked through a cell CSR of F2 (the window's 64x48
//    grid columns are contiguous runs, so a query visits only the keypoints
//    of its cells -- ~60 instead of all n20), keep the kTopK smallest
//    (dist, grid order) keys and the candidate count;
//  2 wave 0: the reference's query loop (ORBmatcher.cpp:510-563) over those
//    lists against the live vMatchedDistance -- a candidate is skipped when
//    vMatchedDistance[i2] <= dist; best = the first kept key, bestDist2 =
//    the next kept key's dist.  64 consecutive queries are resolved at once,
//    one per lane, against the state before the batch; a lane's outcome can
//    only change through a match committed by an EARLIER lane of the batch
//    to an F2 keypoint the lane depends on (vMatchedDistance only decreases,
//    so a skipped entry stays skipped): its best when it matches, its best
//    and second when it fails the ratio test, none when it fails TH_LOW or
//    has no candidate.  The lanes before the first such dependence commit
//    together (their F2 keypoints are distinct), the loop resumes at that
//    lane.  A list that runs out is exact when its last key bounds
//    bestDist2 from below far enough for the ratio test; otherwise the
//    query is re-scanned by the whole wave against the live state (rare).
#ifdef MATCH_STAMPS  // diagnostic build only: phase stamps of block 0 (tools/match_stamps.py)
__device__ unsigned long long g_match_stamps[16];
#define MSTAMP(k)                                                                              \
    do {                                                                                       \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_match_stamps[k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define MSTAMP(k) ((void)0)
#endif

template <int kMaxK0, int kMatchThreads>
__global__ __launch_bounds__(kMatchThreads) void match_init_kernel(
    int more, float minX, float maxX, float minY, float maxY, const orbgpu_keypoint* __restrict__ kps1,
    const uint8_t* __restrict__ desc1, const int* __restrict__ n1p, size_t stride1,
    const orbgpu_keypoint* __restrict__ kps2, const uint8_t* __restrict__ desc2, const int* __restrict__ n2p,
    size_t stride2, float* __restrict__ prev_xy, int window, float nnratio, int flags, int* __restrict__ matches12,
    int* __restrict__ nmatches_out, MatchFirstF1 first) {
    constexpr int kCells = kGC * kGR;
    __shared__ float s_x[kMaxK0], s_y[kMaxK0];
    __shared__ int s_cell[kMaxK0];           // grid cell ix*48+iy, or -1 when not in the grid
    __shared__ int s_mdist[kMaxK0];          // vMatchedDistance
    __shared__ int s_m21[kMaxK0];            // vnMatches21
    constexpr bool kDescHbm = kMaxK0 > kMaxK0Large;  // F2's descriptors stay in HBM (L2-resident)
    // F2's descriptors as four planes (word q of keypoint j at s_d2[q][j]): a
    // 32-byte row per keypoint put every lane's 8-byte read of a random j on
    // the same 4 of the 32 banks (16-way conflicts on every candidate)
    __shared__ unsigned long long s_d2[4][kDescHbm ? 1 : kMaxK0];
    __shared__ int s_m12[kMaxK0];            // vnMatches12 for F1 level-0
    __shared__ float s_px[kMaxK0], s_py[kMaxK0], s_ang1[kMaxK0];  // F1: vbPrevMatched, angle
    __shared__ uint32_t s_top[kMaxK0][kTopK];
    __shared__ int s_ncand[kMaxK0];          // candidates in the window (-1: window off the grid)
    __shared__ short s_cj[kMaxK0];           // F2 index i1 was matched to when the loop reached it, or -1
    __shared__ unsigned short s_cidx[kMaxK0];  // F2 level-0 indices grouped by cell
    __shared__ int s_claim[kMaxK0];          // phase 2: first lane of the batch claiming an F2 keypoint, or 64
    __shared__ int s_cend[kCells];           // cell CSR: end of each cell's run in s_cidx
    __shared__ int s_wsum[kMatchThreads / 64];
    __shared__ int s_hist[kHL];
    __shared__ int s_nm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.x;
    MSTAMP(0);
    // F1 of pair b: frame b of the F1 arrays, or in the stream form (first.kps
    // set) frame b - 1 of them and, for pair 0, the frame before the batch
    // read in place (Tracking's (F_{t-1}, F_t), src/Tracking.cpp:768-769)
    const bool chained = first.kps != nullptr;
    const bool own_first = chained && b == 0;
    const size_t f1 = chained ? (size_t)(b > 0 ? b - 1 : 0) : (size_t)b;
    const orbgpu_keypoint* K1 = own_first ? first.kps : kps1 + f1 * stride1;
    const orbgpu_keypoint* K2 = kps2 + (size_t)b * stride2;
    const uint8_t* D1 = own_first ? first.desc : desc1 + f1 * stride1 * 32;
    const uint8_t* D2 = desc2 + (size_t)b * stride2 * 32;
    const int n1 = own_first ? *first.n : n1p[f1], n2 = n2p[b];
    int* M12 = matches12 + (size_t)b * stride1;
    float* prev = prev_xy ? prev_xy + (size_t)b * stride1 * 2 : nullptr;
    // a larger variant only takes the pairs the previous one handed over
    if (kMaxK0 == kMaxK0Large && nmatches_out[b] != kNeedLarge) return;
    if (kMaxK0 == kMaxK0Huge && nmatches_out[b] != kNeedHuge) return;
    // level-0 counts (the leading octave-0 run of each list, extractor order)
    // counted by the whole block, four loads per thread in flight (a binary
    // search was ten dependent global loads on every thread's path)
    __shared__ int s_l0[2];
    if (tid < 2) s_l0[tid] = 0;
    __syncthreads();
    {
        int c1 = 0, c2 = 0;
        const int nmax = max(n1, n2);
        for (int base = tid; base < nmax; base += 4 * kMatchThreads) {
            int o1[4], o2[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = base + k * kMatchThreads;
                o1[k] = i < n1 ? K1[i].octave : 1;
                o2[k] = i < n2 ? K2[i].octave : 1;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                c1 += o1[k] == 0;
                c2 += o2[k] == 0;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            c1 += __shfl_xor(c1, o, 64);
            c2 += __shfl_xor(c2, o, 64);
        }
        if (lane == 0) {
            atomicAdd(&s_l0[0], c1);
            atomicAdd(&s_l0[1], c2);
        }
    }
    __syncthreads();
    MSTAMP(1);
    const int n10 = s_l0[0], n20 = s_l0[1];
    if (n10 > kMaxK0 || n20 > kMaxK0) {
        // per-pair status: retried by the next variant, or -1 (capacity
        // exceeded); no match is reported for the pair
        for (int i = tid; i < n1; i += kMatchThreads) M12[i] = -1;
        if (tid == 0)
            nmatches_out[b] = !more ? -1 : kMaxK0 == kMaxK0Small ? kNeedLarge : kNeedHuge;
        return;
    }
    const unsigned long long* D2q = reinterpret_cast<const unsigned long long*>(D2);
    auto d2 = [&](int j, int q) -> unsigned long long {
        if constexpr (kDescHbm)
            return D2q[4 * j + q];
        else
            return s_d2[q][j];
    };
    // grid inverses (Frame.cpp:221-224)
    const float invW = __fdiv_rn((float)kGC, __fsub_rn(maxX, minX));
    const float invH = __fdiv_rn((float)kGR, __fsub_rn(maxY, minY));
    for (int c = tid; c < kCells; c += kMatchThreads) s_cend[c] = 0;
    __syncthreads();
    MSTAMP(2);
    for (int j = tid; j < n20; j += kMatchThreads) {
        const float x = K2[j].x, y = K2[j].y;
        s_x[j] = x;
        s_y[j] = y;
        const int px = (int)roundf(__fmul_rn(__fsub_rn(x, minX), invW));
        const int py = (int)roundf(__fmul_rn(__fsub_rn(y, minY), invH));
        const int cell = (px < 0 || px >= kGC || py < 0 || py >= kGR) ? -1 : px * kGR + py;
        s_cell[j] = cell;
        if (cell >= 0) atomicAdd(&s_cend[cell], 1);
        s_mdist[j] = 0x7FFFFFFF;
        s_m21[j] = -1;
        s_claim[j] = 64;
        if (!kDescHbm) {
            const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D2 + (size_t)j * 32);
#pragma unroll
            for (int q = 0; q < 4; ++q) s_d2[q][j] = d[q];
        }
    }
    for (int i = tid; i < n10; i += kMatchThreads) {
        s_m12[i] = -1;
        s_cj[i] = -1;
        s_px[i] = prev ? prev[2 * i] : K1[i].x;
        s_py[i] = prev ? prev[2 * i + 1] : K1[i].y;
        s_ang1[i] = K1[i].angle;
    }
    if (tid < kHL) s_hist[tid] = 0;
    if (tid == 0) s_nm = 0;
    __syncthreads();
    MSTAMP(3);
    {  // exclusive scan of the cell counts: thread t owns cells [12 t, 12 t + 12)
        constexpr int kPer = kCells / kMatchThreads;
        static_assert(kCells % kMatchThreads == 0, "cells per thread");
        int loc[kPer], run = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            loc[k] = run;
            run += s_cend[kPer * tid + k];
        }
        const int incl = wave_incl_scan_dpp(run);
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        int base = incl - run;
        for (int w = 0; w < wave; ++w) base += s_wsum[w];
#pragma unroll
        for (int k = 0; k < kPer; ++k) s_cend[kPer * tid + k] = base + loc[k];  // cell start
        __syncthreads();
        for (int j = tid; j < n20; j += kMatchThreads) {
            const int cell = s_cell[j];
            if (cell >= 0) s_cidx[atomicAdd(&s_cend[cell], 1)] = (unsigned short)j;  // start -> end
        }
        __syncthreads();
    MSTAMP(4);
    }

    const float r = (float)window;
    // GetFeaturesInArea's cell range (Frame.cpp:385-395) for a query at (x, y)
    auto cell_range = [&](float x, float y, int& cx0, int& cx1, int& cy0, int& cy1) {
        cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, minX), r), invW)));
        cx1 = min(kGC - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, minX), r), invW)));
        cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, minY), r), invH)));
        cy1 = min(kGR - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, minY), r), invH)));
        return !(cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0);
    };
    auto in_window = [&](int j, float x, float y, int cx0, int cx1, int cy0, int cy1, int& cell) {
        cell = s_cell[j];
        if (cell < 0) return false;
        const int ix = cell / kGR, iy = cell - ix * kGR;
        if (ix < cx0 || ix > cx1 || iy < cy0 || iy > cy1) return false;
        return fabsf(__fsub_rn(s_x[j], x)) < r && fabsf(__fsub_rn(s_y[j], y)) < r;
    };

    // phase 1: per-query candidate lists (no dependence on the match state).
    // Four lanes per query (an aligned quad): lane sl walks the window's grid
    // columns cx0 + sl, cx0 + sl + 4, ..., keeping its own sorted top-4 and
    // count; the quad then merges by rank through DPP quad permutations (keys
    // are distinct: they carry the keypoint index).  The walk is a chain of
    // dependent LDS reads; one lane per query on four waves ran ~20 columns
    // and ~30 candidates in series (73 k cycles per 1000-feature pair,
    // tools/match_stamps.py); the 1024-thread block runs a pair's ~220
    // queries in one pass of 16 waves, each lane a quarter of a window.
    constexpr int kSub = 4;
    auto quad = [](uint32_t v, auto ctrl) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, decltype(ctrl)::value, 0xF, 0xF, false);
    };
    using QX1 = std::integral_constant<int, 0xB1>;  // quad_perm [1,0,3,2]
    using QX2 = std::integral_constant<int, 0x4E>;  // quad_perm [2,3,0,1]
    using QX3 = std::integral_constant<int, 0x1B>;  // quad_perm [3,2,1,0]
    for (int qbase = 0; qbase < n10; qbase += kMatchThreads / kSub) {
        const int i1 = qbase + tid / kSub, sl = tid % kSub;
        const bool act = i1 < n10;
        int ncand = -1;
        uint32_t top[kTopK];
#pragma unroll
        for (int k = 0; k < kTopK; ++k) top[k] = 0xFFFFFFFFu;
        const float x = act ? s_px[i1] : 0.f, y = act ? s_py[i1] : 0.f;
        int cx0, cx1, cy0, cy1;
        if (act && cell_range(x, y, cx0, cx1, cy0, cy1)) {
            ncand = 0;
            const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D1 + (size_t)i1 * 32);
            const unsigned long long q0 = d[0], q1 = d[1], q2 = d[2], q3 = d[3];
            for (int ix = cx0 + sl; ix <= cx1; ix += kSub) {
                const int c0 = ix * kGR + cy0;
                const int lo = c0 > 0 ? s_cend[c0 - 1] : 0, hi = s_cend[ix * kGR + cy1];
                for (int p = lo; p < hi; ++p) {
                    const int j = s_cidx[p];
                    if (!(fabsf(__fsub_rn(s_x[j], x)) < r && fabsf(__fsub_rn(s_y[j], y)) < r)) continue;
                    const int dist = __popcll(q0 ^ d2(j, 0)) + __popcll(q1 ^ d2(j, 1)) +
                                     __popcll(q2 ^ d2(j, 2)) + __popcll(q3 ^ d2(j, 3));
                    uint32_t key = cand_key(dist, s_cell[j], j);
#pragma unroll
                    for (int k = 0; k < kTopK; ++k) {  // sorted insert
                        const uint32_t lo_k = min(key, top[k]);
                        key = max(key, top[k]);
                        top[k] = lo_k;
                    }
                    ++ncand;
                }
            }
        }
        // quad merge (every lane takes part: DPP reads its quad's lanes)
        uint32_t o1[kTopK], o2[kTopK], o3[kTopK];
#pragma unroll
        for (int k = 0; k < kTopK; ++k) {
            o1[k] = quad(top[k], QX1{});
            o2[k] = quad(top[k], QX2{});
            o3[k] = quad(top[k], QX3{});
        }
        int tot = ncand;  // -1 on all four lanes when the window is off the grid
        tot += (int)quad((uint32_t)tot, QX1{});
        tot += (int)quad((uint32_t)tot, QX2{});
        if (act) {
            if (sl == 0) {
#pragma unroll
                for (int k = 0; k < kTopK; ++k) s_top[i1][k] = 0xFFFFFFFFu;
                s_ncand[i1] = ncand < 0 ? -1 : tot;
            }
#pragma unroll
            for (int k = 0; k < kTopK; ++k) {
                if (top[k] == 0xFFFFFFFFu) continue;
                int rank = k;
#pragma unroll
                for (int t = 0; t < kTopK; ++t) rank += (o1[t] < top[k]) + (o2[t] < top[k]) + (o3[t] < top[k]);
                if (rank < kTopK) s_top[i1][rank] = top[k];
            }
        }
    }
    __syncthreads();
    MSTAMP(5);

    // phase 2 (wave 0, wave-uniform control): batches of 64 queries
    if (wave == 0) {
        auto lds_sync = [] {  // this wave's LDS writes visible to its other lanes
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        };
        int cur = 0;
        while (cur < n10) {
            const int i1 = cur + lane;
            const bool act = i1 < n10;
            const int nc = act ? s_ncand[i1] : 0;
            uint32_t key[kTopK];
            int md[kTopK];
#pragma unroll
            for (int k = 0; k < kTopK; ++k) key[k] = act ? s_top[i1][k] : 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < kTopK; ++k) md[k] = key[k] != 0xFFFFFFFFu ? s_mdist[key_j(key[k])] : 0;
            const int nk = min(nc, kTopK);
            uint32_t best = 0xFFFFFFFFu, second = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < kTopK; ++k) {
                if (k >= nk || second != 0xFFFFFFFFu) continue;
                if (md[k] <= key_dist(key[k])) continue;  // vMatchedDistance[i2] <= dist
                if (best == 0xFFFFFFFFu) best = key[k]; else second = key[k];
            }
            // 0 no match, 1 match, 2 needs the exact re-scan
            int state = 0;
            if (nc > 0) {
                if (best == 0xFFFFFFFFu) {
                    state = nc > kTopK ? 2 : 0;
                } else {
                    const int bd = key_dist(best);
                    if (bd > kThLow) state = 0;
                    else if (second != 0xFFFFFFFFu) state = (float)bd < __fmul_rn((float)key_dist(second), nnratio) ? 1 : 0;
                    else if (nc <= kTopK) state = (float)bd < __fmul_rn((float)0x7FFFFFFF, nnratio) ? 1 : 0;
                    // bestDist2 >= the last listed key's dist: enough when it passes the ratio test
                    else state = (float)bd < __fmul_rn((float)key_dist(key[kTopK - 1]), nnratio) ? 1 : 2;
                }
            }
            const int claim = state == 1 ? key_j(best) : -1;
            if (claim >= 0) atomicMin(&s_claim[claim], lane);
            lds_sync();
            // F2 keypoints this lane's outcome depends on (see above)
            int dep0 = -1, dep1 = -1;
            if (state == 1) {
                dep0 = claim;
            } else if (state == 0 && best != 0xFFFFFFFFu && key_dist(best) <= kThLow) {
                dep0 = key_j(best);  // failed the ratio test: best and second decide it
                dep1 = second != 0xFFFFFFFFu ? key_j(second) : -1;
            }
            const bool dep = (dep0 >= 0 && s_claim[dep0] < lane) || (dep1 >= 0 && s_claim[dep1] < lane);
            const unsigned long long stop = __ballot(act && (dep || state == 2));
            const int ncommit = stop ? (int)__builtin_ctzll(stop) : min(64, n10 - cur);
            if (lane < ncommit && state == 1) {  // distinct F2 keypoints: no ordering among these lanes
                const int prev21 = s_m21[claim];
                if (prev21 >= 0) s_m12[prev21] = -1;  // a match of an earlier batch is taken over
                s_m12[i1] = claim;
                s_m21[claim] = i1;
                s_mdist[claim] = key_dist(best);
                s_cj[i1] = (short)claim;
            }
            if (claim >= 0) s_claim[claim] = 64;
            lds_sync();
            if (ncommit > 0) {
                cur += ncommit;
                continue;
            }
            // the batch's first query needs the exact re-scan against the live state
            {
                const int q = cur;
                const float x = s_px[q], y = s_py[q];
                int cx0, cx1, cy0, cy1;
                cell_range(x, y, cx0, cx1, cy0, cy1);
                const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D1 + (size_t)q * 32);
                const unsigned long long q0 = d[0], q1 = d[1], q2 = d[2], q3 = d[3];
                unsigned long long lbest = ~0ull;
                int second2 = 0x7FFFFFFF;
                for (int j = lane; j < n20; j += 64) {
                    int cell;
                    if (!in_window(j, x, y, cx0, cx1, cy0, cy1, cell)) continue;
                    const int dist = __popcll(q0 ^ d2(j, 0)) + __popcll(q1 ^ d2(j, 1)) +
                                     __popcll(q2 ^ d2(j, 2)) + __popcll(q3 ^ d2(j, 3));
                    if (s_mdist[j] <= dist) continue;
                    const unsigned long long k64 = ((unsigned long long)dist << 32) | ((unsigned)cell << 16) | (unsigned)j;
                    if (k64 < lbest) {
                        if (lbest != ~0ull) second2 = min(second2, (int)(lbest >> 32));
                        lbest = k64;
                    } else {
                        second2 = min(second2, dist);
                    }
                }
                const unsigned long long wbest = wave_min_u64(lbest);
                const int contrib = lbest == wbest ? second2 : (lbest == ~0ull ? 0x7FFFFFFF : (int)(lbest >> 32));
                const int best2 = wave_min_i(contrib);
                if (wbest != ~0ull) {
                    const int bestDist = (int)(wbest >> 32), bidx = (int)(wbest & 0xFFFF);
                    if (bestDist <= kThLow && (float)bestDist < __fmul_rn((float)best2, nnratio) && lane == 0) {
                        const int prev21 = s_m21[bidx];
                        if (prev21 >= 0) s_m12[prev21] = -1;
                        s_m12[q] = bidx;
                        s_m21[bidx] = q;
                        s_mdist[bidx] = bestDist;
                        s_cj[q] = (short)bidx;
                    }
                }
                lds_sync();
                cur += 1;
            }
        }
    }
    __syncthreads();
    MSTAMP(6);
    if (flags & ORBGPU_MATCH_CHECK_ORI) {
        // rotHist (ORBmatcher.cpp:541-552): one entry per query matched when the loop reached it
        const float factor =
            (flags & ORBGPU_MATCH_ANNOTATED_HISTO) ? __fdiv_rn(1.0f, (float)kHL) : __fdiv_rn((float)kHL, 360.0f);
        for (int i = tid; i < n10; i += kMatchThreads) {
            const int j = s_cj[i];
            int bin = -1;
            if (j >= 0) {
                float rot = __fsub_rn(s_ang1[i], K2[j].angle);
                if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                bin = (int)roundf(__fmul_rn(rot, factor));
                if (bin == kHL) bin = 0;
                atomicAdd(&s_hist[bin], 1);
            }
            s_cj[i] = (short)bin;
        }
        __syncthreads();
        // ComputeThreeMaxima (ORBmatcher.cpp:1792-1833), then cull other bins
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHL; ++i) {
            const int s = s_hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < __fmul_rn(0.1f, (float)max1)) ind3 = -1;
        for (int i = tid; i < n10; i += kMatchThreads) {
            const int bin = s_cj[i];
            if (bin >= 0 && bin != ind1 && bin != ind2 && bin != ind3) s_m12[i] = -1;
        }
        __syncthreads();
    }
    int nmatches = 0;
    for (int i = tid; i < n1; i += kMatchThreads) {
        const int m = i < n10 ? s_m12[i] : -1;
        M12[i] = m;
        if (m >= 0) {
            ++nmatches;
            if (prev) { prev[2 * i] = s_x[m]; prev[2 * i + 1] = s_y[m]; }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nmatches += __shfl_xor(nmatches, o, 64);
    if (lane == 0) atomicAdd(&s_nm, nmatches);
    __syncthreads();
    if (tid == 0) nmatches_out[b] = s_nm;
    MSTAMP(8);
}

__global__ __launch_bounds__(256) void hamming_pairs_kernel(const uint8_t* __restrict__ a,
                                                            const uint8_t* __restrict__ b, int n,
                                                            int* __restrict__ dist) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const ulonglong4 x = reinterpret_cast<const ulonglong4*>(a)[i];
    const ulonglong4 y = reinterpret_cast<const ulonglong4*>(b)[i];
    dist[i] = __popcll(x.x ^ y.x) + __popcll(x.y ^ y.y) + __popcll(x.z ^ y.z) + __popcll(x.w ^ y.w);
}

// Threads per pair block.  Phase 2 runs on one wave while the block's other
// waves keep their slots, so a batch that fills the chip (the stream bench:
// the matcher beside the next batch's extraction) takes the block size
// ORBGPU_MATCH_THREADS names (256, 512 or 1024; default kBatchThreads) and
// leaves more of the chip to the kernels beside it; a few pairs (the
// drop-in's one) take 1024 threads, the shortest phase 1.
constexpr int kChipFill = 256;
int match_batch_threads() {
    const char* s = std::getenv("ORBGPU_MATCH_THREADS");
    const int v = s ? std::atoi(s) : kBatchThreads;
    return v == 256 || v == 512 || v == 1024 ? v : kBatchThreads;
}

bool match_tiny_enabled() {
    static const bool v = [] {  // read once per process (A/B runs set it per process)
        const char* s = std::getenv("ORBGPU_MATCH_TINY");
        return !s || std::atoi(s) != 0;
    }();
    return v;
}

template <int kMaxK0, int kThreads>
hipError_t launch_variant(int batch, int more, float minX, float maxX, float minY, float maxY,
                          const orbgpu_keypoint* kps1, const uint8_t* desc1, const int* n1, size_t stride1,
                          const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2, size_t stride2,
                          float* prev_xy, int window, float nnratio, int flags, int* matches12, int* nmatches,
                          hipStream_t stream, MatchFirstF1 first) {
    hipLaunchKernelGGL((match_init_kernel<kMaxK0, kThreads>), dim3(batch), dim3(kThreads), 0, stream, more, minX, maxX,
                       minY, maxY, kps1, desc1, n1, stride1, kps2, desc2, n2, stride2, prev_xy, window, nnratio, flags,
                       matches12, nmatches, first);
    return hipGetLastError();
}

}  // namespace

#ifdef MATCH_STAMPS
extern "C" int orbgpu_debug_match_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_match_stamps), sizeof(g_match_stamps)) == hipSuccess ? 0 : -2;
}
#endif

hipError_t launch_hamming_pairs(const uint8_t* a, const uint8_t* b, int n, int* dist, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(hamming_pairs_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, b, n, dist);
    return hipGetLastError();
}

hipError_t launch_match_init(int batch, float minX, float maxX, float minY, float maxY,
                             const orbgpu_keypoint* kps1, const uint8_t* desc1, const int* n1, size_t stride1,
                             const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2, size_t stride2,
                             float* prev_xy, int window, float nnratio, int flags,
                             int* matches12, int* nmatches, hipStream_t stream, size_t level0_bound,
                             MatchFirstF1 first) {
    // small variant for every pair, then the larger ones for the pairs handed
    // over (a no-op block per other pair, which still waits for a CU with the
    // variant's LDS free); a larger variant is launched only when a frame's
    // level-0 keypoints can exceed the previous limit: bounded by its capacity
    // (stride), or by level0_bound when the caller knows it (the host form
    // counts them; a batch caller passes its extractor's level-0 output
    // capacity).  The last variant launched reports a pair above its limit as -1.
    const size_t cap = level0_bound ? level0_bound : (stride1 > stride2 ? stride1 : stride2);
    const int more_large = cap > (size_t)kMaxK0Small, more_huge = cap > (size_t)kMaxK0Large;
    const int threads = batch >= kChipFill ? match_batch_threads() : 1024;
    hipError_t e;
#define ORBGPU_MATCH_ARGS                                                                                         \
    minX, maxX, minY, maxY, kps1, desc1, n1, stride1, kps2, desc2, n2, stride2, prev_xy, window, nnratio, flags, \
        matches12, nmatches, stream, first
    // a level-0 bound of at most 256 keypoints (1000 features: 220 slots): the 256 variant alone,
    // ~38 KB of LDS per block instead of ~62 KB, so the matcher's blocks take less room beside
    // the extraction kernels they overlap (ORBGPU_MATCH_TINY=0: the 512 variant)
    if (cap <= (size_t)kMaxK0Tiny && batch >= kChipFill && match_tiny_enabled()) {
        if (threads == 256)
            e = launch_variant<kMaxK0Tiny, 256>(batch, 0, ORBGPU_MATCH_ARGS);
        else if (threads == 512)
            e = launch_variant<kMaxK0Tiny, 512>(batch, 0, ORBGPU_MATCH_ARGS);
        else
            e = launch_variant<kMaxK0Tiny, 1024>(batch, 0, ORBGPU_MATCH_ARGS);
        return e;
    }
    if (threads == 256)
        e = launch_variant<kMaxK0Small, 256>(batch, more_large, ORBGPU_MATCH_ARGS);
    else if (threads == 512)
        e = launch_variant<kMaxK0Small, 512>(batch, more_large, ORBGPU_MATCH_ARGS);
    else
        e = launch_variant<kMaxK0Small, 1024>(batch, more_large, ORBGPU_MATCH_ARGS);
    if (e == hipSuccess && more_large) e = launch_variant<kMaxK0Large, 1024>(batch, more_huge, ORBGPU_MATCH_ARGS);
    if (e == hipSuccess && more_huge) e = launch_variant<kMaxK0Huge, 1024>(batch, 0, ORBGPU_MATCH_ARGS);
#undef ORBGPU_MATCH_ARGS
    return e;
}

}  // namespace orbgpu
