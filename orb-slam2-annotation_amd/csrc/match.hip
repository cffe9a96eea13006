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
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "../../include/orbgpu.h"

namespace orbgpu {

namespace {

// Level-0 keypoints per frame held in LDS.  The 512 variant (45 KB of LDS)
// covers nfeatures <= 2350; pairs above it are handed to the 1024 variant
// (89 KB: the 2x-features initialisation extractor of KITTI mono,
// Tracking.cpp:149, has ~870 at level 0); above 1024 a pair reports -1.
constexpr int kMaxK0Small = 512, kMaxK0Large = 1024;
constexpr int kNeedLarge = -2;  // nmatches sentinel: the pair waits for the large variant
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

// number of leading octave-0 keypoints
__device__ int level0_count(const orbgpu_keypoint* k, int n) {
    int lo = 0, hi = n;  // first index with octave != 0
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (k[mid].octave == 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

constexpr int kMatchThreads = 256;
constexpr int kTopK = 4;  // best candidate keys kept per query by the parallel phase

// (dist, grid order) of a candidate as one ordered key: dist <= 256 (9 bits),
// cell = ix * 48 + iy < 3072 (12 bits), level-0 index < 1024 (10 bits)
constexpr int kKeyJBits = 10;
constexpr uint32_t kKeyJMask = (1u << kKeyJBits) - 1;
__device__ inline uint32_t cand_key(int dist, int cell, int j) {
    return ((uint32_t)dist << (12 + kKeyJBits)) | ((uint32_t)cell << kKeyJBits) | (uint32_t)j;
}
__device__ inline int key_dist(uint32_t key) { return (int)(key >> (12 + kKeyJBits)); }
__device__ inline int key_j(uint32_t key) { return (int)(key & kKeyJMask); }

// Two phases per frame pair (one 256-thread block):
//  1 parallel, one thread per F1 query: scan the level-0 F2 keypoints (same
//    j for every lane: LDS broadcasts), keep the kTopK smallest (dist, grid
//    order) keys of the candidates in the query's window, and their count;
//  2 sequential, wave 0: the reference's query loop (ORBmatcher.cpp:510-563)
//    over those lists -- a candidate is skipped when vMatchedDistance[i2] <=
//    dist (state of the loop so far); best = first kept key, bestDist2 = the
//    next kept key's dist.  A list is exact while it holds all candidates or
//    both values are found inside it; otherwise the query is re-scanned by
//    the whole wave against the live state (rare).
template <int kMaxK0>
__global__ __launch_bounds__(kMatchThreads) void match_init_kernel(
    float minX, float maxX, float minY, float maxY, const orbgpu_keypoint* __restrict__ kps1,
    const uint8_t* __restrict__ desc1, const int* __restrict__ n1p, size_t stride1,
    const orbgpu_keypoint* __restrict__ kps2, const uint8_t* __restrict__ desc2, const int* __restrict__ n2p,
    size_t stride2, float* __restrict__ prev_xy, int window, float nnratio, int flags, int* __restrict__ matches12,
    int* __restrict__ nmatches_out) {
    __shared__ float s_x[kMaxK0], s_y[kMaxK0];
    __shared__ int s_cell[kMaxK0];           // grid cell ix*48+iy, or -1 when not in the grid
    __shared__ int s_mdist[kMaxK0];          // vMatchedDistance
    __shared__ int s_m21[kMaxK0];            // vnMatches21
    __shared__ unsigned long long s_d2[kMaxK0][4];
    __shared__ int s_m12[kMaxK0];            // vnMatches12 for F1 level-0
    __shared__ float s_px[kMaxK0], s_py[kMaxK0], s_ang1[kMaxK0];  // F1: vbPrevMatched, angle
    __shared__ uint32_t s_top[kMaxK0][kTopK];
    __shared__ int s_ncand[kMaxK0];          // candidates in the window (-1: window off the grid)
    __shared__ short s_cj[kMaxK0];           // F2 index i1 was matched to when the loop reached it, or -1
    __shared__ int s_hist[kHL];
    __shared__ int s_nm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.x;
    const orbgpu_keypoint* K1 = kps1 + (size_t)b * stride1;
    const orbgpu_keypoint* K2 = kps2 + (size_t)b * stride2;
    const uint8_t* D1 = desc1 + (size_t)b * stride1 * 32;
    const uint8_t* D2 = desc2 + (size_t)b * stride2 * 32;
    const int n1 = n1p[b], n2 = n2p[b];
    int* M12 = matches12 + (size_t)b * stride1;
    float* prev = prev_xy ? prev_xy + (size_t)b * stride1 * 2 : nullptr;
    const bool large = kMaxK0 == kMaxK0Large;
    // the large variant only takes the pairs the small one handed over
    if (large && nmatches_out[b] != kNeedLarge) return;
    const int n10 = level0_count(K1, n1), n20 = level0_count(K2, n2);
    if (n10 > kMaxK0 || n20 > kMaxK0) {
        // per-pair status: kNeedLarge (retried by the large variant) or -1
        // (capacity exceeded); no match is reported for the pair
        for (int i = tid; i < n1; i += kMatchThreads) M12[i] = -1;
        if (tid == 0) nmatches_out[b] = large ? -1 : kNeedLarge;
        return;
    }
    // grid inverses (Frame.cpp:221-224)
    const float invW = __fdiv_rn((float)kGC, __fsub_rn(maxX, minX));
    const float invH = __fdiv_rn((float)kGR, __fsub_rn(maxY, minY));
    for (int j = tid; j < n20; j += kMatchThreads) {
        const float x = K2[j].x, y = K2[j].y;
        s_x[j] = x;
        s_y[j] = y;
        const int px = (int)roundf(__fmul_rn(__fsub_rn(x, minX), invW));
        const int py = (int)roundf(__fmul_rn(__fsub_rn(y, minY), invH));
        s_cell[j] = (px < 0 || px >= kGC || py < 0 || py >= kGR) ? -1 : px * kGR + py;
        s_mdist[j] = 0x7FFFFFFF;
        s_m21[j] = -1;
        const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D2 + (size_t)j * 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) s_d2[j][q] = d[q];
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

    // phase 1: per-query candidate lists (no dependence on the match state)
    for (int i1 = tid; i1 < n10; i1 += kMatchThreads) {
        const float x = s_px[i1], y = s_py[i1];
        int cx0, cx1, cy0, cy1;
        int ncand = -1;
        uint32_t top[kTopK];
#pragma unroll
        for (int k = 0; k < kTopK; ++k) top[k] = 0xFFFFFFFFu;
        if (cell_range(x, y, cx0, cx1, cy0, cy1)) {
            ncand = 0;
            const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D1 + (size_t)i1 * 32);
            const unsigned long long q0 = d[0], q1 = d[1], q2 = d[2], q3 = d[3];
            for (int j = 0; j < n20; ++j) {
                int cell;
                if (!in_window(j, x, y, cx0, cx1, cy0, cy1, cell)) continue;
                const int dist = __popcll(q0 ^ s_d2[j][0]) + __popcll(q1 ^ s_d2[j][1]) +
                                 __popcll(q2 ^ s_d2[j][2]) + __popcll(q3 ^ s_d2[j][3]);
                uint32_t key = cand_key(dist, cell, j);
#pragma unroll
                for (int k = 0; k < kTopK; ++k) {  // sorted insert
                    const uint32_t lo = min(key, top[k]);
                    key = max(key, top[k]);
                    top[k] = lo;
                }
                ++ncand;
            }
        }
#pragma unroll
        for (int k = 0; k < kTopK; ++k) s_top[i1][k] = top[k];
        s_ncand[i1] = ncand;
    }
    __syncthreads();

    // phase 2: the sequential query loop (wave 0; wave-uniform control).  The
    // lists of 64 queries at a time are read into lanes and taken from there
    // with readlane, so a query costs one LDS round trip (vMatchedDistance of
    // its listed candidates) plus the commit; the rotation bins are computed
    // after the loop from the F2 index each query was matched to when the
    // loop reached it (the reference pushes i1 into rotHist at that moment,
    // and a later steal does not remove it), in parallel.
    if (wave == 0) {
        for (int base = 0; base < n10; base += 64) {
            const int qi = base + lane;
            int l_nc = 0;
            uint32_t l_top[kTopK];
#pragma unroll
            for (int k = 0; k < kTopK; ++k) l_top[k] = 0xFFFFFFFFu;
            if (qi < n10) {
                l_nc = s_ncand[qi];
#pragma unroll
                for (int k = 0; k < kTopK; ++k) l_top[k] = s_top[qi][k];
            }
            const int cnt = min(64, n10 - base);
            for (int u = 0; u < cnt; ++u) {
                const int i1 = base + u;
                const int ncand = __builtin_amdgcn_readlane(l_nc, u);
                if (ncand <= 0) continue;  // window off the grid, or no candidate in it
                uint32_t key[kTopK];
                int md[kTopK];
#pragma unroll
                for (int k = 0; k < kTopK; ++k) key[k] = __builtin_amdgcn_readlane(l_top[k], u);
#pragma unroll
                for (int k = 0; k < kTopK; ++k) md[k] = key[k] != 0xFFFFFFFFu ? s_mdist[key_j(key[k])] : 0;
                uint32_t best = 0xFFFFFFFFu;
                int best2 = 0x7FFFFFFF;
                bool have2 = false;
                const int nk = min(ncand, kTopK);
#pragma unroll
                for (int k = 0; k < kTopK; ++k) {
                    if (k >= nk || have2) continue;
                    const int dist = key_dist(key[k]);
                    if (md[k] <= dist) continue;
                    if (best == 0xFFFFFFFFu) {
                        best = key[k];
                    } else {
                        best2 = dist;
                        have2 = true;
                    }
                }
                if (!have2 && ncand > kTopK) {
                    // the list ran out: exact re-scan against the live state
                    const float x = s_px[i1], y = s_py[i1];
                    int cx0, cx1, cy0, cy1;
                    cell_range(x, y, cx0, cx1, cy0, cy1);
                    const unsigned long long* d = reinterpret_cast<const unsigned long long*>(D1 + (size_t)i1 * 32);
                    const unsigned long long q0 = d[0], q1 = d[1], q2 = d[2], q3 = d[3];
                    unsigned long long lbest = ~0ull;
                    int second = 0x7FFFFFFF;
                    for (int j = lane; j < n20; j += 64) {
                        int cell;
                        if (!in_window(j, x, y, cx0, cx1, cy0, cy1, cell)) continue;
                        const int dist = __popcll(q0 ^ s_d2[j][0]) + __popcll(q1 ^ s_d2[j][1]) +
                                         __popcll(q2 ^ s_d2[j][2]) + __popcll(q3 ^ s_d2[j][3]);
                        if (s_mdist[j] <= dist) continue;
                        const unsigned long long k64 = ((unsigned long long)dist << 32) | ((unsigned)cell << 16) | (unsigned)j;
                        if (k64 < lbest) {
                            if (lbest != ~0ull) second = min(second, (int)(lbest >> 32));
                            lbest = k64;
                        } else {
                            second = min(second, dist);
                        }
                    }
                    const unsigned long long wbest = wave_min_u64(lbest);
                    const int contrib = lbest == wbest ? second : (lbest == ~0ull ? 0x7FFFFFFF : (int)(lbest >> 32));
                    best2 = wave_min_i(contrib);
                    best = wbest == ~0ull ? 0xFFFFFFFFu
                                          : cand_key((int)(wbest >> 32), (int)((wbest >> 16) & 0xFFFF), (int)(wbest & 0xFFFF));
                }
                if (best == 0xFFFFFFFFu) continue;  // no usable candidate
                const int bestDist = key_dist(best);
                const int bidx = key_j(best);
                if (bestDist <= kThLow && (float)bestDist < __fmul_rn((float)best2, nnratio)) {
                    if (lane == 0) {
                        const int prev21 = s_m21[bidx];
                        if (prev21 >= 0) s_m12[prev21] = -1;
                        s_m12[i1] = bidx;
                        s_m21[bidx] = i1;
                        s_mdist[bidx] = bestDist;
                        s_cj[i1] = (short)bidx;
                    }
                    // wave-local LDS ordering for the next query's reads
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
            }
        }
    }
    __syncthreads();
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

}  // namespace

hipError_t launch_hamming_pairs(const uint8_t* a, const uint8_t* b, int n, int* dist, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(hamming_pairs_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, b, n, dist);
    return hipGetLastError();
}

hipError_t launch_match_init(int batch, float minX, float maxX, float minY, float maxY,
                             const orbgpu_keypoint* kps1, const uint8_t* desc1, const int* n1, size_t stride1,
                             const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2, size_t stride2,
                             float* prev_xy, int window, float nnratio, int flags,
                             int* matches12, int* nmatches, hipStream_t stream) {
    // small variant for every pair, then the large one for the pairs it
    // handed over (a no-op block per pair otherwise)
    hipLaunchKernelGGL(match_init_kernel<kMaxK0Small>, dim3(batch), dim3(kMatchThreads), 0, stream, minX, maxX, minY,
                       maxY, kps1, desc1, n1, stride1, kps2, desc2, n2, stride2, prev_xy, window, nnratio, flags,
                       matches12, nmatches);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(match_init_kernel<kMaxK0Large>, dim3(batch), dim3(kMatchThreads), 0, stream, minX, maxX, minY,
                       maxY, kps1, desc1, n1, stride1, kps2, desc2, n2, stride2, prev_xy, window, nnratio, flags,
                       matches12, nmatches);
    return hipGetLastError();
}

}  // namespace orbgpu
