// pnp.hip -- PnPsolver's RANSAC loop (src/PnPsolver.cpp:203-349) for a batch
// of solvers (one per relocalisation candidate keyframe), in two launches:
//   1  pnp_hyp_kernel: 16 lanes per hypothesis (four per wave) run EPnP
//      (epnp_wave.h) on its minimal set of 4 correspondences and score it
//      (CheckInliers :352-386, the group's lanes over the correspondences)
//      -- speculative, all n_hyp of every solver;
//   2  pnp_score_kernel, one 256-thread block per solver, chunks of 256
//      hypothesis counts in LDS: the whole block replays the
//      reference's loop body in iteration order: a hypothesis with
//      inliers >= minInliers becomes the best if it beats it (its mask is
//      written by all threads), and Refine() (:303-349: EPnP over all best
//      inliers, then CheckInliers) runs on wave 0 (the inlier list by an
//      ordered ballot compaction, EPnP with the correspondences over the 64
//      lanes); the first refinement
//      with more than minInliers inliers ends the call.  Refine() of an
//      unchanged best is deterministic, so it is evaluated once per best.
// Parity with the CPU oracle is to a stated pose tolerance
// (tests/test_pnp.py): the reference's cvSVD is restated with Jacobi
// methods and the null space of a minimal set is only defined up to a basis.
#include "../../include/orbgpu_ransac.h"
#include "epnp.h"
#include "epnp_wave.h"
#include "ransac_kernels.h"

namespace orbgpu {

namespace {

constexpr int kThreads = 256;

#ifdef EPNP_STAMPS  // diagnostic build only (tools/epnp_stamps.py)
// [0]: EPnP phases of block (0, 0) group 0 of pnp_hyp_kernel; [1]: the first
// Refine of solver 0; [2]: pnp_score_kernel phases of solver 0
__device__ unsigned long long g_epnp_stamps[3][32];
#define SCORE_T(k)                                                                      \
    do {                                                                                \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_epnp_stamps[2][k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define SCORE_T(k) ((void)0)
#endif
constexpr int kChunk = 256;  // hypothesis counts staged in LDS at a time

struct HypPose {
    double R[9], t[3];
    int inliers;  // CheckInliers count, by the group that solved it
    int pad;
};

struct SampleSrc {  // the minimal set of one hypothesis
    const float* P3;
    const float* P2;
    const int* idx;
    __device__ int count() const { return 4; }
    __device__ void get(int i, double* pw, double& u, double& v) const {
        const int k = idx[i];
        pw[0] = P3[3 * k];
        pw[1] = P3[3 * k + 1];
        pw[2] = P3[3 * k + 2];
        u = P2[2 * k];
        v = P2[2 * k + 1];
    }
};

struct ListSrc {  // Refine(): the best inliers in index order
    const float* P3;
    const float* P2;
    const int* list;
    int n;
    __device__ int count() const { return n; }
    __device__ void get(int i, double* pw, double& u, double& v) const {
        const int k = list[i];
        pw[0] = P3[3 * k];
        pw[1] = P3[3 * k + 1];
        pw[2] = P3[3 * k + 2];
        u = P2[2 * k];
        v = P2[2 * k + 1];
    }
};

// PnPsolver::CheckInliers (:352-386): camera coordinates in float from the
// double pose, projection in double, squared error in float
__device__ inline bool pnp_inlier(const HypPose& H, const epnp::Camera& cam, const float* P3, const float* P2,
                                  float maxerr) {
    const double x = P3[0], y = P3[1], z = P3[2];
    const float Xc = (float)(H.R[0] * x + H.R[1] * y + H.R[2] * z + H.t[0]);
    const float Yc = (float)(H.R[3] * x + H.R[4] * y + H.R[5] * z + H.t[1]);
    const float invZc = (float)(1 / (H.R[6] * x + H.R[7] * y + H.R[8] * z + H.t[2]));
    const double ue = cam.uc + cam.fu * (double)Xc * (double)invZc;
    const double ve = cam.vc + cam.fv * (double)Yc * (double)invZc;
    const float dx = (float)((double)P2[0] - ue), dy = (float)((double)P2[1] - ve);
    const float e2 = dx * dx + dy * dy;
    return e2 < maxerr;
}

__device__ inline epnp::Camera camera_of(const orbgpu_pnp_problem& P) {
    return epnp::Camera{(double)P.fu, (double)P.fv, (double)P.uc, (double)P.vc};
}

__device__ inline void pose_to_tcw(const HypPose& H, float* T) {  // Rcw/tcw convertTo(CV_32F) into eye(4)
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = (float)H.R[3 * i + j];
        T[4 * i + 3] = (float)H.t[i];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

__global__ __launch_bounds__(64) void pnp_hyp_kernel(const orbgpu_pnp_problem* __restrict__ probs,
                                                     const float* __restrict__ P3g, const float* __restrict__ P2g,
                                                     const float* __restrict__ errg, const int* __restrict__ samples,
                                                     HypPose* __restrict__ hyps) {
    __shared__ double s_ep[4][epnp::kWaveScratch];
    const orbgpu_pnp_problem& P = probs[blockIdx.y];
    const int lane = threadIdx.x, g = lane >> 4, r = lane & 15;
    const int h = blockIdx.x * 4 + g;
    if (h >= P.n_hyp) return;  // the whole 16-lane group leaves together
    const size_t slot = (size_t)P.sample_offset + h;
    SampleSrc src{P3g + 3 * (size_t)P.offset, P2g + 2 * (size_t)P.offset, samples + 4 * slot};
    const epnp::Camera cam = camera_of(P);
    epnp::Pose pose;
#ifdef EPNP_STAMPS
    unsigned long long* st = (blockIdx.x == 0 && blockIdx.y == 0 && g == 0) ? g_epnp_stamps[0] : nullptr;
#else
    unsigned long long* st = nullptr;
#endif
    epnp::compute_pose_group<16>(src, cam, pose, r, s_ep[g], st);
    HypPose H;
    for (int k = 0; k < 9; ++k) H.R[k] = pose.R[k];
    for (int k = 0; k < 3; ++k) H.t[k] = pose.t[k];
    // CheckInliers (:352-386) of this hypothesis by the same group: every
    // hypothesis of the batch is scored here, in parallel, so the replay in
    // pnp_score_kernel only reads the counts
    const float* P3 = P3g + 3 * (size_t)P.offset;
    const float* P2 = P2g + 2 * (size_t)P.offset;
    const float* E = errg + P.offset;
    int cnt = 0;
    for (int i = r; i < P.n; i += 16) cnt += pnp_inlier(H, cam, P3 + 3 * i, P2 + 2 * i, E[i]);
    cnt += __shfl_xor(cnt, 1, 16);
    cnt += __shfl_xor(cnt, 2, 16);
    cnt += __shfl_xor(cnt, 4, 16);
    cnt += __shfl_xor(cnt, 8, 16);
    H.inliers = cnt;
    H.pad = 0;
    if (r == 0) hyps[slot] = H;
}

__global__ __launch_bounds__(kThreads) void pnp_score_kernel(const orbgpu_pnp_problem* __restrict__ probs,
                                                             const HypPose* __restrict__ hyps,
                                                             const float* __restrict__ P3g,
                                                             const float* __restrict__ P2g,
                                                             const float* __restrict__ errg,
                                                             int* __restrict__ lists,
                                                             orbgpu_pnp_result* __restrict__ results,
                                                             uint8_t* __restrict__ best_mask,
                                                             uint8_t* __restrict__ refined_mask) {
    __shared__ int s_cnt[kChunk];
    __shared__ int s_state[6];  // best, best_hyp, found, consumed, refine_tried, refined_inliers
    __shared__ HypPose s_ref;
    __shared__ double s_ep[epnp::kWaveScratch];
    __shared__ double s_jac[JacobiLds<12, 12>::kDoubles];
    const orbgpu_pnp_problem P = probs[blockIdx.x];
    const HypPose* HP = hyps + P.sample_offset;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* P3 = P3g + 3 * (size_t)P.offset;
    const float* P2 = P2g + 2 * (size_t)P.offset;
    const float* E = errg + P.offset;
    uint8_t* BM = best_mask + P.offset;
    int* list = lists + P.offset;
    const epnp::Camera cam = camera_of(P);
    if (tid == 0) {
        s_state[0] = P.best_inliers;
        s_state[1] = -1;
        s_state[2] = 0;
        s_state[3] = 0;
        s_state[4] = 0;  // Refine() of the incoming best not evaluated yet
        s_state[5] = 0;
    }
    __syncthreads();
    SCORE_T(0);
    for (int base = 0; base < P.n_hyp && !s_state[2]; base += kChunk) {
        const int nh = min(kChunk, P.n_hyp - base);
        for (int h = tid; h < nh; h += kThreads) s_cnt[h] = HP[base + h].inliers;  // scored by pnp_hyp_kernel
        __syncthreads();
        for (int h = 0; h < nh; ++h) {  // block-uniform replay of the loop body (:224-299)
            const int c = s_cnt[h];
            if (c < P.min_inliers) continue;
            if (c > s_state[0]) {  // new best: its inlier mask
                const HypPose& H = HP[base + h];
                for (int i = tid; i < P.n; i += kThreads) BM[i] = pnp_inlier(H, cam, P3 + 3 * i, P2 + 2 * i, E[i]);
                __syncthreads();
                SCORE_T(1);
                if (tid == 0) {
                    s_state[0] = c;
                    s_state[1] = base + h;
                    s_state[4] = 0;
                }
                __syncthreads();
            }
            if (!s_state[4]) {  // Refine() with the current best inliers
                if (wave == 0) {
                    int m = 0;  // the best inliers in index order (ordered ballot compaction)
                    for (int b0 = 0; b0 < P.n; b0 += 64) {
                        const int i = b0 + lane;
                        const bool in = i < P.n && BM[i];
                        const unsigned long long bal = __ballot(in);
                        if (in) list[m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] = i;
                        m += __popcll(bal);
                    }
                    __builtin_amdgcn_s_waitcnt(0);  // the list is in memory before any lane reads it
                    __builtin_amdgcn_wave_barrier();
                    SCORE_T(2);
                    ListSrc src{P3, P2, list, m};
                    epnp::Pose pose;
#ifdef EPNP_STAMPS
                    unsigned long long* st = (blockIdx.x == 0 && !s_state[3]) ? g_epnp_stamps[1] : nullptr;
#else
                    unsigned long long* st = nullptr;
#endif
                    if (m > 0) epnp::compute_pose_group<64>(src, cam, pose, lane, s_ep, st, s_jac);
                    if (lane == 0) {
                        for (int k = 0; k < 9; ++k) s_ref.R[k] = m > 0 ? pose.R[k] : 0.0;
                        for (int k = 0; k < 3; ++k) s_ref.t[k] = m > 0 ? pose.t[k] : 0.0;
                    }
                }
                __syncthreads();
                SCORE_T(3);
                int cnt = 0;
                for (int i = tid; i < P.n; i += kThreads) {
                    const bool in = pnp_inlier(s_ref, cam, P3 + 3 * i, P2 + 2 * i, E[i]);
                    refined_mask[P.offset + i] = in;
                    cnt += in;
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                if (tid == 0) s_state[5] = 0;
                __syncthreads();
                if (lane == 0) atomicAdd(&s_state[5], cnt);
                __syncthreads();
                if (tid == 0) {
                    s_state[4] = 1;
                    if (s_state[5] > P.min_inliers) {
                        s_state[2] = 1;
                        s_state[3] = base + h + 1;
                    }
                }
                __syncthreads();
                if (s_state[2]) break;
            }
        }
        __syncthreads();
    }
    SCORE_T(4);
    if (tid == 0) {
        orbgpu_pnp_result& R = results[blockIdx.x];
        R.found = s_state[2];
        R.consumed = s_state[2] ? s_state[3] : P.n_hyp;
        R.best_inliers = s_state[0];
        R.best_hyp = s_state[1];
        R.refined_inliers = s_state[2] ? s_state[5] : 0;
        if (s_state[1] >= 0) pose_to_tcw(HP[s_state[1]], R.best_Tcw);
        if (s_state[2]) pose_to_tcw(s_ref, R.refined_Tcw);
    }
}

// qr_solve_6x4 on its own, one thread per problem (debug ABI, tests)
__global__ void qr_solve_kernel(const double* A, const double* b, double* X, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a[24], bb[6], x[4];
    for (int k = 0; k < 24; ++k) a[k] = A[(size_t)i * 24 + k];
    for (int k = 0; k < 6; ++k) bb[k] = b[(size_t)i * 6 + k];
    for (int k = 0; k < 4; ++k) x[k] = X[(size_t)i * 4 + k];
    epnp::qr_solve_6x4(a, bb, x);
    for (int k = 0; k < 4; ++k) X[(size_t)i * 4 + k] = x[k];
}

}  // namespace

size_t pnp_hyp_bytes() { return sizeof(HypPose); }

}  // namespace orbgpu

extern "C" int orbgpu_debug_qr_solve_6x4_device(const double* A, const double* b, double* X, int n, void* stream) {
    if (n <= 0) return 0;
    if (!A || !b || !X) return -1;
    hipLaunchKernelGGL(orbgpu::qr_solve_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, A, b, X, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

namespace orbgpu {

#ifdef EPNP_STAMPS
extern "C" int orbgpu_debug_epnp_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_epnp_stamps), sizeof(g_epnp_stamps)) == hipSuccess ? 0 : -2;
}
#endif

hipError_t launch_pnp_ransac(int batch, const orbgpu_pnp_problem* probs, int max_hyp, const float* P3,
                             const float* P2, const float* maxerr, const int* samples, void* hyps, int* lists,
                             orbgpu_pnp_result* results, uint8_t* best_mask, uint8_t* refined_mask,
                             hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (max_hyp > 0)
        hipLaunchKernelGGL(pnp_hyp_kernel, dim3((max_hyp + 3) / 4, batch), dim3(64), 0, stream, probs, P3, P2,
                           maxerr, samples, static_cast<HypPose*>(hyps));
    hipLaunchKernelGGL(pnp_score_kernel, dim3(batch), dim3(kThreads), 0, stream, probs,
                       static_cast<const HypPose*>(hyps), P3, P2, maxerr, lists, results, best_mask, refined_mask);
    return hipGetLastError();
}

}  // namespace orbgpu
