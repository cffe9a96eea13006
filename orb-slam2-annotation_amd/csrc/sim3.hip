// sim3.hip -- Sim3Solver's RANSAC inner loop (Sim3Solver.cpp:147-221) for a
// batch of solvers, in two launches:
//
//   1  sim3_hyp_kernel: one thread per hypothesis of the whole batch solves
//      Horn's closed form for its minimal triplet (ComputeSim3, :225-327):
//      centroids, M = Pr2 Pr1^T, the 4x4 quaternion matrix N, its dominant
//      eigenvector (cyclic Jacobi), angle-axis -> Rodrigues, scale, T12, T21;
//   2  sim3_score_kernel, one 256-thread block per solver, chunks of 64
//      hypotheses: the 4 waves score them, lanes over correspondences --
//      both reprojection errors against the truncated 9.210*sigma^2
//      thresholds (CheckInliers, :331-358, Project :378-400), counted with
//      ballot + popcount -- then one lane replays the sequential acceptance
//      over the chunk in iteration order: best update on inliers >= best,
//      stop at the first hypothesis with inliers > minInliers.
// Work past the stopping hypothesis is speculative and discarded, so the
// observable result is the reference loop's.
//
// Arithmetic follows the reference's cv::Mat expressions: float storage,
// products of small float matrices accumulated in double (OpenCV's
// GEMMSingleMul<float,double>), quaternion matrix entries formed in float,
// angle-axis and Rodrigues in double.  Parity with the CPU oracle is to a
// stated tolerance (tests/test_ransac.py), not bitwise: cos/sin/atan2 of
// the device math library and of glibc may differ in the last ulp.
#include "../../include/orbgpu_ransac.h"
#include "orbgpu_internal.h"
#include "ransac_kernels.h"
#include "sim3_device.h"

namespace orbgpu {

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 64;
using namespace sim3dev;

// one thread per hypothesis (speculative: all n_hyp of every solver; the
// scorer below stops at the reference's exit point).  Hypothesis h of
// problem b lives in slot sample_offset + h, like its triplet.
__global__ __launch_bounds__(64) void sim3_hyp_kernel(const orbgpu_sim3_problem* __restrict__ probs,
                                                      const float* __restrict__ X1g, const float* __restrict__ X2g,
                                                      const int* __restrict__ samples, Hyp* __restrict__ hyps) {
    const orbgpu_sim3_problem& P = probs[blockIdx.y];
    const int h = blockIdx.x * 64 + threadIdx.x;
    if (h >= P.n_hyp) return;
    const float* X1 = X1g + 3 * (size_t)P.offset;
    const float* X2 = X2g + 3 * (size_t)P.offset;
    const int* S = samples + 3 * ((size_t)P.sample_offset + h);
    float A[3][3], B[3][3];
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) {
            A[k][i] = X1[3 * S[k] + i];
            B[k][i] = X2[3 * S[k] + i];
        }
    compute_sim3(A, B, P.fix_scale != 0, hyps[(size_t)P.sample_offset + h]);
}

__global__ __launch_bounds__(kThreads) void sim3_score_kernel(const orbgpu_sim3_problem* __restrict__ probs,
                                                              const Hyp* __restrict__ hyps,
                                                              const float* __restrict__ X1g,
                                                              const float* __restrict__ X2g,
                                                              const float* __restrict__ e1g,
                                                              const float* __restrict__ e2g,
                                                              orbgpu_sim3_result* __restrict__ results,
                                                              uint8_t* __restrict__ inliers) {
    __shared__ int s_cnt[kChunk];
    __shared__ int s_state[4];  // best, best_hyp, found, consumed
    const orbgpu_sim3_problem P = probs[blockIdx.x];
    const Hyp* HP = hyps + P.sample_offset;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* X1 = X1g + 3 * (size_t)P.offset;
    const float* X2 = X2g + 3 * (size_t)P.offset;
    const float* E1 = e1g + P.offset;
    const float* E2 = e2g + P.offset;
    if (tid == 0) {
        s_state[0] = P.best_inliers;
        s_state[1] = -1;
        s_state[2] = 0;
        s_state[3] = 0;
    }
    __syncthreads();
    for (int base = 0; base < P.n_hyp; base += kChunk) {
        const int nh = min(kChunk, P.n_hyp - base);
        for (int h = wave; h < nh; h += kThreads / 64) {  // score
            const Hyp& H = HP[base + h];
            int cnt = 0;
            for (int i = lane; i < P.n; i += 64) {
                const bool in = is_inlier(H, P.K1, P.K2, X1 + 3 * i, X2 + 3 * i, E1[i], E2[i]);
                cnt += __popcll(__ballot(in));
            }
            if (lane == 0) s_cnt[h] = cnt;
        }
        __syncthreads();
        if (tid == 0) {  // the reference's acceptance, in iteration order
            int best = s_state[0], bh = s_state[1], found = 0, consumed = base + nh;
            for (int h = 0; h < nh; ++h) {
                const int c = s_cnt[h];
                if (c >= best) {
                    best = c;
                    bh = base + h;
                    if (c > P.min_inliers) {
                        found = 1;
                        consumed = base + h + 1;
                        break;
                    }
                }
            }
            s_state[0] = best;
            s_state[1] = bh;
            s_state[2] = found;
            s_state[3] = consumed;
        }
        __syncthreads();
        if (s_state[2]) break;
    }
    const int bh = s_state[1];
    if (bh >= 0) {
        const Hyp& H = HP[bh];
        for (int i = tid; i < P.n; i += kThreads)
            inliers[P.offset + i] = is_inlier(H, P.K1, P.K2, X1 + 3 * i, X2 + 3 * i, E1[i], E2[i]) ? 1 : 0;
    }
    if (tid == 0) {
        orbgpu_sim3_result& R = results[blockIdx.x];
        R.found = s_state[2];
        R.consumed = P.n_hyp > 0 ? s_state[3] : 0;
        R.best_inliers = s_state[0];
        R.best_hyp = bh;
        if (bh >= 0) {
            const Hyp& H = HP[bh];
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) R.T12[4 * i + j] = H.sR[3 * i + j];
                R.T12[4 * i + 3] = H.t[i];
                R.t12[i] = H.t[i];
            }
            R.T12[12] = R.T12[13] = R.T12[14] = 0.f;
            R.T12[15] = 1.f;
            for (int k = 0; k < 9; ++k) R.R12[k] = H.R[k];
            R.s12 = H.s;
        }
    }
}

}  // namespace

size_t sim3_hyp_bytes() { return sizeof(Hyp); }

hipError_t launch_sim3_ransac(int batch, const orbgpu_sim3_problem* probs, int max_hyp, const float* X1,
                              const float* X2, const float* e1, const float* e2, const int* samples, void* hyps,
                              orbgpu_sim3_result* results, uint8_t* inliers, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (max_hyp > 0)
        hipLaunchKernelGGL(sim3_hyp_kernel, dim3((max_hyp + 63) / 64, batch), dim3(64), 0, stream, probs, X1, X2,
                           samples, static_cast<Hyp*>(hyps));
    hipLaunchKernelGGL(sim3_score_kernel, dim3(batch), dim3(kThreads), 0, stream, probs,
                       static_cast<const Hyp*>(hyps), X1, X2, e1, e2, results, inliers);
    return hipGetLastError();
}

}  // namespace orbgpu
