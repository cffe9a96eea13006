// loop.hip -- LoopClosing::ComputeSim3 (src/LoopClosing.cpp:273-420) after
// SearchByBoW: the Sim3Solver constructors of all candidates, then the
// round-robin RANSAC of every query (include/orbgpu_loop.h).
//
//   sim3_setup_kernel    one 256-thread block per candidate: the ctor's loop
//                        over vpMatched12 (Sim3Solver.cpp:54-99) as an
//                        order-preserving compaction (ballot prefix sums),
//                        camera-frame points Rcw*Xw + tcw with
//                        double-accumulated products, truncated error bounds.
//   compute_sim3_kernel  one 512-thread block per query.  Lane 0 lays out
//                        the reference's hypothesis order -- rounds of
//                        iterate(5) over the live candidates, 3 RandomInt
//                        swap-remove draws per hypothesis from the query's
//                        glibc stream -- for a window of 256 hypotheses; every
//                        thread solves one of them (Horn, sim3_device.h), the
//                        8 waves score them (lanes over correspondences,
//                        ballot + popcount), and lane 0 replays the acceptance
//                        in stream order (best on >=, return on > minInliers).
//                        The first return ends the query; hypotheses past it
//                        were speculative and are discarded.
#include "../../include/orbgpu_loop.h"
#include "host_common.h"
#include "orbgpu_internal.h"
#include "sim3_device.h"

namespace orbgpu {

namespace {

using namespace sim3dev;

constexpr int kThreads = 256;       // sim3_setup_kernel
#ifndef ORBGPU_SIM3_THREADS
#define ORBGPU_SIM3_THREADS 512
#endif
constexpr int kQThreads = ORBGPU_SIM3_THREADS;  // compute_sim3_kernel: 8 scoring waves, 2 per SIMD
constexpr int kWin = 256;  // hypotheses solved and scored per window
constexpr int kMaxC = ORBGPU_LOOP_MAX_CANDIDATES;

struct Workspace {  // SoA, candidate c at c * stride
    float* X1;      // 3 per correspondence
    float* X2;
    float* e1;
    float* e2;
    int* idx1;
    float2* P1;     // mvP1im1 / mvP2im2: FromCameraToImage of X1 / X2 (the ctor's, Sim3Solver.cpp:97-98)
    float2* P2;
};

__host__ __device__ inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

__host__ __device__ inline Workspace carve(void* base, int n_cand, int stride) {
    const size_t n = (size_t)n_cand * stride;
    char* p = static_cast<char*>(base);
    Workspace w;
    w.X1 = reinterpret_cast<float*>(p);
    p += align256(n * 12);
    w.X2 = reinterpret_cast<float*>(p);
    p += align256(n * 12);
    w.e1 = reinterpret_cast<float*>(p);
    p += align256(n * 4);
    w.e2 = reinterpret_cast<float*>(p);
    p += align256(n * 4);
    w.idx1 = reinterpret_cast<int*>(p);
    p += align256(n * 4);
    w.P1 = reinterpret_cast<float2*>(p);
    p += align256(n * 8);
    w.P2 = reinterpret_cast<float2*>(p);
    return w;
}

size_t workspace_bytes(int n_cand, int stride) {
    const size_t n = (size_t)(n_cand > 0 ? n_cand : 1) * (stride > 0 ? stride : 1);
    return 2 * align256(n * 12) + 3 * align256(n * 4) + 2 * align256(n * 8);
}

// mvnMaxError = 9.210*sigma^2 kept in a vector<size_t> (Sim3Solver.cpp:92-93)
__device__ inline float max_error(float sigma2) { return (float)(unsigned long long)(9.210 * (double)sigma2); }

__global__ __launch_bounds__(kThreads) void sim3_setup_kernel(const orbgpu_sim3_candidate* __restrict__ cands,
                                                              const orbgpu_loop_keyframe* __restrict__ kfs,
                                                              const int* __restrict__ match12, int stride,
                                                              const int* __restrict__ nmatches, int min_matches,
                                                              Workspace ws, int* __restrict__ n_corr) {
    __shared__ int s_wave[kThreads / 64];
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nmatches[c] < min_matches) {  // LoopClosing.cpp:314-318: no solver is built
        if (tid == 0) n_corr[c] = -1;
        return;
    }
    const orbgpu_sim3_candidate cd = cands[c];
    const orbgpu_loop_keyframe& K1 = kfs[cd.kf1];
    const orbgpu_loop_keyframe& K2 = kfs[cd.kf2];
    const int* row = match12 + (size_t)c * stride;
    const size_t o = (size_t)c * stride;
    const int n1 = min(K1.n, stride);
    int base = 0;
    for (int s = 0; s < n1; s += kThreads) {
        const int i1 = s + tid;
        int i2 = -1;
        if (i1 < n1) {
            i2 = row[i1];
            if (i2 >= K2.n || (i2 >= 0 && !(K1.mp_valid[i1] && K2.mp_valid[i2]))) i2 = -1;
        }
        const bool ok = i2 >= 0;
        const unsigned long long m = __ballot(ok);
        if (lane == 0) s_wave[wave] = __popcll(m);
        __syncthreads();
        int before = base;
        for (int w = 0; w < wave; ++w) before += s_wave[w];
        if (ok) {
            const int j = before + (int)__popcll(m & ((1ull << lane) - 1));
            float Xw[3], Xc[3];
            float u, v;  // mvP1im1 / mvP2im2: FromCameraToImage (the per-hypothesis test's fixed half)
            for (int k = 0; k < 3; ++k) Xw[k] = K1.mp_world[3 * (size_t)i1 + k];
            for (int k = 0; k < 3; ++k) Xc[k] = gemv_row(&K1.Rcw[3 * k], Xw) + K1.tcw[k];
            for (int k = 0; k < 3; ++k) ws.X1[3 * (o + j) + k] = Xc[k];
            to_image(K1.K, Xc, u, v);
            ws.P1[o + j] = make_float2(u, v);
            for (int k = 0; k < 3; ++k) Xw[k] = K2.mp_world[3 * (size_t)i2 + k];
            for (int k = 0; k < 3; ++k) Xc[k] = gemv_row(&K2.Rcw[3 * k], Xw) + K2.tcw[k];
            for (int k = 0; k < 3; ++k) ws.X2[3 * (o + j) + k] = Xc[k];
            to_image(K2.K, Xc, u, v);
            ws.P2[o + j] = make_float2(u, v);
            ws.e1[o + j] = max_error(K1.sigma2[K1.octave[i1]]);
            ws.e2[o + j] = max_error(K2.sigma2[K2.octave[i2]]);
            ws.idx1[o + j] = i1;
        }
        for (int w = 0; w < kThreads / 64; ++w) base += s_wave[w];
        __syncthreads();
    }
    if (tid == 0) n_corr[c] = base;
}

// glibc random_r TYPE_3 step (csrc/ransac.cpp restates the same generator):
// returns the raw sum written into the state; rand() is raw >> 1
__device__ inline uint32_t rand_next_raw(int32_t* r, int& f, int& b) {
    const uint32_t val = (uint32_t)r[f] + (uint32_t)r[b];
    r[f] = (int32_t)val;
    if (++f >= 31) {
        f = 0;
        ++b;
    } else if (++b >= 31) {
        b = 0;
    }
    return val;
}

// DUtils::Random::RandomInt(0, d-1)
__device__ inline int random_below(int32_t v, int d) {
    return (int)(((double)v / ((double)2147483647 + 1.0)) * d);
}

__global__ __launch_bounds__(kQThreads) void compute_sim3_kernel(
    const orbgpu_compute_sim3_query* __restrict__ queries, const orbgpu_sim3_candidate* __restrict__ cands,
    const orbgpu_loop_keyframe* __restrict__ kfs, int stride, Workspace ws, const int* __restrict__ n_corr,
    orbgpu_sim3_ransac_params prm, orbgpu_compute_sim3_result* __restrict__ results,
    orbgpu_sim3_candidate_state* __restrict__ states, uint8_t* __restrict__ inliers) {
    __shared__ Hyp s_hyp[kWin];
    __shared__ Hyp s_best[kMaxC];
    __shared__ int s_slot_c[kWin], s_slot_r[kWin], s_trip[kWin][3], s_cnt[kWin];
    __shared__ int c_n[kMaxC], c_max[kMaxC], c_its[kMaxC], c_best[kMaxC], c_sched[kMaxC];
    __shared__ unsigned char c_live[kMaxC];  // still scheduled (not discarded)
    __shared__ int32_t s_r[31];
    // the stream at the current window's start and the raw values its layout
    // drew: the state after exactly the consumed draws is rebuilt from these
    // (the last 31 raw values are the generator's whole state)
    __shared__ int32_t s_snap[31], s_gen[3 * kWin];
    __shared__ int s_nslots, s_done, s_matched, s_round, s_total;
    __shared__ float s_K[kMaxC][8];  // each candidate's K1, K2 (fx, fy, cx, cy): no dependent loads per hypothesis
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const orbgpu_compute_sim3_query Q = queries[q];
    const int nc = Q.n_cand;
    const int c0 = Q.first_cand;
    const int ipc = prm.iterations_per_call;
    if (tid < nc) {  // Sim3Solver::SetRansacParameters (Sim3Solver.cpp:111-141)
        const orbgpu_sim3_candidate cd = cands[c0 + tid];
        for (int k = 0; k < 4; ++k) {
            s_K[tid][k] = kfs[cd.kf1].K[k];
            s_K[tid][4 + k] = kfs[cd.kf2].K[k];
        }
        const int N = n_corr[c0 + tid];
        c_n[tid] = N;
        int max_its = 0;
        if (N >= 0) {
            const float eps = (float)prm.min_inliers / (float)N;
            int n_it;
            if (prm.min_inliers == N) {
                n_it = 1;
            } else {
                const double v = ceil(log(1.0 - prm.probability) / log(1.0 - pow((double)eps, 3.0)));
                // an out-of-range double -> int conversion is INT_MIN on x86 (cvttsd2si)
                n_it = (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (int)0x80000000;
            }
            max_its = max(1, min(n_it, prm.max_iterations));
        }
        c_max[tid] = max_its;
        c_its[tid] = 0;
        c_best[tid] = 0;
        c_sched[tid] = 0;
        // no solver (N < 0), or iterate() returns bNoMore at once (N < minInliers, :151-156)
        c_live[tid] = (N >= 0 && N >= prm.min_inliers) ? 1 : 0;
    }
    if (tid == 0) {
        for (int k = 0; k < 31; ++k) s_r[k] = Q.rng.r[k];
        s_done = 0;
        s_matched = -1;
        s_round = -1;
        s_total = 0;
    }
    __syncthreads();
    int rf = Q.rng.f, rb = Q.rng.b;        // lane 0's stream indices
    int snap_f = rf, snap_b = rb, snap_total = 0;  // lane 0: the current window's start
    int cur_round = 0, cur_c = 0, cur_j = 0;  // lane 0's schedule cursor
    bool sched_end = false;
    // windows grow 32, 64, .., kWin: most queries return within a few
    // hypotheses, so the first windows stay small (less speculative work)
    int win = 32;
    while (true) {
        if (tid == 0) {  // lay out the next window in the reference's order
            for (int k = 0; k < 31; ++k) s_snap[k] = s_r[k];
            snap_f = rf;
            snap_b = rb;
            snap_total = s_total;
            int n = 0;
            while (n < win && !sched_end) {
                if (cur_c == nc) {  // next round of `while (nCandidates > 0 && !bMatch)`
                    bool any = false;
                    for (int c = 0; c < nc; ++c) any |= c_live[c] != 0;
                    if (!any) {
                        sched_end = true;
                        break;
                    }
                    cur_c = 0;
                    ++cur_round;
                }
                const int c = cur_c;
                if (!c_live[c]) {
                    ++cur_c;
                    continue;
                }
                const int k = min(ipc, c_max[c] - c_sched[c]);  // iterations of this iterate() call
                for (; cur_j < k && n < win; ++cur_j, ++n) {
                    // vAvailableIndices = mvAllIndices; 3 x RandomInt + swap-remove (Sim3Solver.cpp:172-183)
                    const int N = c_n[c];
                    int pos[2], val[2], nmod = 0;
                    for (int d = 0; d < 3; ++d) {
                        const int size = N - d;
                        const uint32_t raw = rand_next_raw(s_r, rf, rb);
                        s_gen[3 * n + d] = (int32_t)raw;
                        const int r = random_below((int32_t)(raw >> 1), size);
                        int idx = r;  // vAvailableIndices[r] after the earlier swaps
                        for (int m = nmod - 1; m >= 0; --m)
                            if (pos[m] == r) {
                                idx = val[m];
                                break;
                            }
                        int back = size - 1;  // vAvailableIndices.back()
                        for (int m = nmod - 1; m >= 0; --m)
                            if (pos[m] == size - 1) {
                                back = val[m];
                                break;
                            }
                        s_trip[n][d] = idx;
                        if (d < 2) {
                            pos[nmod] = r;
                            val[nmod] = back;
                            ++nmod;
                        }
                    }
                    s_slot_c[n] = c;
                    s_slot_r[n] = cur_round;
                }
                if (cur_j == k) {  // the call is laid out completely
                    cur_j = 0;
                    c_sched[c] += k;
                    if (c_sched[c] >= c_max[c]) c_live[c] = 0;  // bNoMore -> vbDiscarded (:349-353)
                    ++cur_c;
                }
            }
            s_nslots = n;
        }
        __syncthreads();
        const int ns = s_nslots;
        if (ns == 0) break;
        if (tid < ns) {  // ComputeSim3 for one hypothesis
            const int c = s_slot_c[tid];
            const size_t o = (size_t)(c0 + c) * stride;
            float A[3][3], B[3][3];
            for (int k = 0; k < 3; ++k)
                for (int i = 0; i < 3; ++i) {
                    A[k][i] = ws.X1[3 * (o + s_trip[tid][k]) + i];
                    B[k][i] = ws.X2[3 * (o + s_trip[tid][k]) + i];
                }
            compute_sim3(A, B, prm.fix_scale != 0, s_hyp[tid]);
        }
        __syncthreads();
        // CheckInliers: a wave takes the hypotheses 2p and 2p + 1 (pairs p = wave,
        // wave + 8, ..); consecutive hypotheses are mostly one candidate's iterate(5)
        // run, and then one pass over its correspondences tests both (each
        // correspondence loaded once).  Four correspondences per lane in flight (one
        // wave per SIMD here: the test's loads and FP64 chains are latency bound, so
        // independent work is what hides them); indices past N are clamped and masked.
        for (int p = wave; 2 * p < ns; p += kQThreads / 64) {
            const int h0 = 2 * p, h1 = 2 * p + 1;
            const int c = s_slot_c[h0];
            const bool both = h1 < ns && s_slot_c[h1] == c;  // wave-uniform
            auto check = [&](int h, int hb, bool two) {  // hypotheses h (and hb when two) of candidate s_slot_c[h]
                const int cc = s_slot_c[h];
                const float* K1 = s_K[cc];
                const float* K2 = s_K[cc] + 4;
                const size_t o = (size_t)(c0 + cc) * stride;
                const int N = c_n[cc];
                int cnt = 0, cntb = 0;
                for (int i0 = lane; i0 < N; i0 += 256) {
                    bool in[4], inb[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = min(i0 + 64 * u, N - 1);
                        const float* X1 = ws.X1 + 3 * (o + i);
                        const float* X2 = ws.X2 + 3 * (o + i);
                        const float2 p1 = ws.P1[o + i], p2 = ws.P2[o + i];
                        const float e1 = ws.e1[o + i], e2 = ws.e2[o + i];
                        in[u] = is_inlier_pre(s_hyp[h], K1, K2, X1, X2, p1, p2, e1, e2);
                        inb[u] = two && is_inlier_pre(s_hyp[hb], K1, K2, X1, X2, p1, p2, e1, e2);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool live = i0 + 64 * u < N;
                        cnt += __popcll(__ballot(in[u] && live));
                        if (two) cntb += __popcll(__ballot(inb[u] && live));
                    }
                }
                if (lane == 0) {
                    s_cnt[h] = cnt;
                    if (two) s_cnt[hb] = cntb;
                }
            };
            if (both) {
                check(h0, h1, true);
            } else {
                check(h0, h0, false);
                if (h1 < ns) check(h1, h1, false);
            }
        }
        __syncthreads();
        if (tid == 0) {  // the reference's acceptance, in stream order (Sim3Solver.cpp:199-212)
            for (int h = 0; h < ns; ++h) {
                const int c = s_slot_c[h], cnt = s_cnt[h];
                ++c_its[c];
                ++s_total;
                if (cnt >= c_best[c]) {
                    c_best[c] = cnt;
                    s_best[c] = s_hyp[h];
                    if (cnt > prm.min_inliers) {
                        s_matched = c;
                        s_round = s_slot_r[h];
                        s_done = 1;
                        break;
                    }
                }
            }
        }
        __syncthreads();
        if (s_done) break;
        win = min(2 * win, kWin);
    }
    __syncthreads();
    const int mc = s_matched;
    if (mc >= 0) {  // mvbBestInliers of the returning candidate
        const float* K1 = s_K[mc];
        const float* K2 = s_K[mc] + 4;
        const size_t o = (size_t)(c0 + mc) * stride;
        for (int i = tid; i < c_n[mc]; i += kQThreads)
            inliers[o + i] = is_inlier_pre(s_best[mc], K1, K2, ws.X1 + 3 * (o + i), ws.X2 + 3 * (o + i), ws.P1[o + i],
                                           ws.P2[o + i], ws.e1[o + i], ws.e2[o + i]) ? 1 : 0;
    }
    if (tid < nc) {
        orbgpu_sim3_candidate_state& S = states[c0 + tid];
        S.n = c_n[tid];
        S.max_iterations = c_max[tid];
        S.iterations = c_its[tid];
        S.best_inliers = c_best[tid];
        S.discarded = (c_n[tid] < prm.min_inliers || (tid != mc && c_its[tid] >= c_max[tid])) ? 1 : 0;
        S.pad = 0;
    }
    if (tid == 0) {
        orbgpu_compute_sim3_result& R = results[q];
        R.matched = mc;
        R.round = s_round;
        R.hypotheses = s_total;
        R.draws = 3 * s_total;
        R.pad = 0;
        R.n_inliers = mc >= 0 ? c_best[mc] : 0;
        if (mc >= 0) {
            const Hyp& H = s_best[mc];
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) R.T12[4 * i + j] = H.sR[3 * i + j];
                R.T12[4 * i + 3] = H.t[i];
                R.t12[i] = H.t[i];
            }
            R.T12[12] = R.T12[13] = R.T12[14] = 0.f;
            R.T12[15] = 1.f;
            for (int k = 0; k < 9; ++k) R.R12[k] = H.R[k];
            R.s12 = H.s;
        } else {
            for (int k = 0; k < 16; ++k) R.T12[k] = 0.f;
            for (int k = 0; k < 9; ++k) R.R12[k] = 0.f;
            for (int k = 0; k < 3; ++k) R.t12[k] = 0.f;
            R.s12 = 0.f;
        }
        // the stream after exactly the consumed draws: the last window's start
        // state with its first K raw values written at slots snap_f, snap_f+1, ..
        // (mod 31), and both indices advanced by K
        const int K = 3 * (s_total - snap_total);
        for (int k = 0; k < 31; ++k) R.rng_after.r[k] = s_snap[k];
        for (int j = max(0, K - 31); j < K; ++j) R.rng_after.r[(snap_f + j) % 31] = s_gen[j];
        R.rng_after.f = (snap_f + K) % 31;
        R.rng_after.b = (snap_b + K) % 31;
    }
}

}  // namespace

}  // namespace orbgpu

using namespace orbgpu;

extern "C" {

size_t orbgpu_sim3_setup_workspace_bytes(int n_cand, int match_stride) {
    return workspace_bytes(n_cand, match_stride);
}

const int* orbgpu_sim3_corr_kf1_slots(const void* d_workspace, int n_cand, int match_stride, int c) {
    if (!d_workspace || c < 0 || c >= n_cand || match_stride <= 0) return nullptr;
    return carve(const_cast<void*>(d_workspace), n_cand, match_stride).idx1 + (size_t)c * match_stride;
}

int orbgpu_sim3_setup_batch_device(int n_cand, const orbgpu_sim3_candidate* d_cands,
                                   const orbgpu_loop_keyframe* d_kfs, const int* d_match12, int match_stride,
                                   const int* d_nmatches, int min_matches, void* d_workspace, int* d_n_corr,
                                   void* stream) {
    if (n_cand < 0 || match_stride <= 0 ||
        (n_cand > 0 && (!d_cands || !d_kfs || !d_match12 || !d_nmatches || !d_workspace || !d_n_corr)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (n_cand == 0) return ORBGPU_OK;
    if (int rc = check_device()) return rc;
    (void)hipGetLastError();
    hipLaunchKernelGGL(sim3_setup_kernel, dim3(n_cand), dim3(kThreads), 0, (hipStream_t)stream, d_cands, d_kfs,
                       d_match12, match_stride, d_nmatches, min_matches, carve(d_workspace, n_cand, match_stride),
                       d_n_corr);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_compute_sim3_batch_device(int n_queries, const orbgpu_compute_sim3_query* d_queries,
                                     int n_cand, const orbgpu_sim3_candidate* d_cands, const orbgpu_loop_keyframe* d_kfs,
                                     int match_stride, const void* d_workspace, const int* d_n_corr,
                                     orbgpu_sim3_ransac_params params, orbgpu_compute_sim3_result* d_results,
                                     orbgpu_sim3_candidate_state* d_cand_states, uint8_t* d_inliers,
                                     void* stream) {
    if (n_queries < 0 || n_cand < 0 || match_stride <= 0 || params.iterations_per_call < 1 || params.max_iterations < 1 ||
        params.min_inliers < 0 || !(params.probability > 0.0 && params.probability < 1.0) ||
        (n_queries > 0 && (!d_queries || !d_cands || !d_kfs || !d_workspace || !d_n_corr || !d_results ||
                           !d_cand_states || !d_inliers)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (n_queries == 0) return ORBGPU_OK;
    if (int rc = check_device()) return rc;
    (void)hipGetLastError();
    hipLaunchKernelGGL(compute_sim3_kernel, dim3(n_queries), dim3(kQThreads), 0, (hipStream_t)stream, d_queries,
                       d_cands, d_kfs, match_stride, carve(const_cast<void*>(d_workspace), n_cand, match_stride), d_n_corr,
                       params, d_results, d_cand_states, d_inliers);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

}  // extern "C"
