// init_models.hip -- the model hypotheses of the monocular Initializer
// (src/Initializer.cpp:55-388) for all RANSAC iterations in two launches
// (include/orbgpu_init.h, orbgpu_init_hypotheses_batch_device):
//
//   init_normalize_kernel  Normalize (:965-1015) of both frames' keypoints:
//                          one lane per (frame, axis) runs the reference's
//                          sequential float sums (mean, then mean absolute
//                          deviation), the block writes the normalised points;
//                          also the match list (u1, v1, u2, v2) the scorers read.
//   init_models_kernel     one wave per (iteration, model): lanes 0..15 build
//                          the rows of the DLT matrix A in float as ComputeH21
//                          (:292-330, 16 x 9) / ComputeF21 (:332-388, 8 x 9 +
//                          zero rows) build it, in LDS; its right singular
//                          vector of the smallest singular value
//                          (cv::SVDecomp's vt.row(8)) by one-sided (Hestenes)
//                          Jacobi in double with the five disjoint column
//                          pairs of each round-robin round on five 8-lane
//                          groups (jacobi_lds.h; numerically null columns take
//                          no rotation -- the 8 x 9 F system always has one);
//                          then lane 0 does, for F, the rank-2 projection
//                          (w(2) = 0), the de-normalisation T2inv*Hn*T1 /
//                          T2t*Fn*T1 and H12 = H21.inv() with OpenCV's float
//                          3x3 products (double accumulation) and 3x3
//                          closed-form inverse.  (Round 2 ran one thread per
//                          hypothesis with the 16 x 9 and 9 x 9 doubles in
//                          scratch: 5.1 ms per 200 + 200 hypotheses; round 3
//                          first ran 16 lanes per model with the rows on the
//                          lanes, jacobi_group.h: 92 us.)
// The SVDs are restated (OpenCV's Jacobi SVD in float is not reproducible
// here), so H/F match the oracle to a tolerance; CheckHomography /
// CheckFundamental (init.hip) then score them bit-exactly.
#include <hip/hip_runtime.h>

#include "../../include/orbgpu_init.h"
#include "epnp.h"
#include "group_sum.h"
#include "jacobi_group.h"
#include "jacobi_lds.h"
#include "host_common.h"

namespace {

constexpr int kNormThreads = 256;
constexpr int kNormChunk = 2048;  // keypoints per frame staged in LDS at a time (2 x 16 KB)

// Normalize (Initializer.cpp:965-1015).  work layout (floats):
//   [0, 2 n1)            normalised mvKeys1
//   [2 n1, 2 n1 + 2 n2)  normalised mvKeys2
//   then T1 (9), T2 (9)
__global__ __launch_bounds__(kNormThreads) void init_normalize_kernel(const float* __restrict__ kp1, int n1,
                                                                      const float* __restrict__ kp2, int n2,
                                                                      const int* __restrict__ pairs, int nm,
                                                                      float* __restrict__ work,
                                                                      float4* __restrict__ pts) {
    __shared__ float s_mean[4], s_scale[4];
    __shared__ float2 s_kp[2][kNormChunk];
    const int tid = threadIdx.x;
    // lane = (frame, axis) runs the reference's sequential float sums (mean,
    // then mean absolute deviation) over LDS; the block stages the keypoints
    // chunk by chunk with coalesced loads (a lane walking them in HBM paid one
    // dependent memory round trip per keypoint: 177 us for 2 x 2000)
    const int fr = (tid >> 1) & 1, ax = tid & 1;
    const int n = fr ? n2 : n1;
    const int nmax = n1 > n2 ? n1 : n2;
    float mean = 0.f, acc = 0.f;
    for (int pass = 0; pass < 2; ++pass) {
        for (int base = 0; base < nmax; base += kNormChunk) {
            __syncthreads();  // the previous chunk is consumed
            // eight loads per thread in flight before any store (a copy loop
            // waited one memory latency per element)
            for (int i0 = tid; i0 < 2 * kNormChunk; i0 += 8 * kNormThreads) {
                float2 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int i = i0 + k * kNormThreads;
                    const int f = i / kNormChunk, j = i - f * kNormChunk, idx = base + j;
                    const int nf = f ? n2 : n1;
                    v[k] = (i < 2 * kNormChunk && idx < nf) ? reinterpret_cast<const float2*>(f ? kp2 : kp1)[idx]
                                                            : make_float2(0.f, 0.f);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int i = i0 + k * kNormThreads;
                    const int f = i / kNormChunk, j = i - f * kNormChunk;
                    if (i < 2 * kNormChunk && base + j < (f ? n2 : n1)) s_kp[f][j] = v[k];
                }
            }
            __syncthreads();
            if (tid < 4) {
                // 32 keypoints per step: their LDS reads issued ahead of the dependent adds
                const int cnt = min(kNormChunk, n - base);
                const float* colv = reinterpret_cast<const float*>(s_kp[fr]) + ax;
                int i = 0;
                if (pass == 0) {
                    for (; i + 32 <= cnt; i += 32) {
                        float v[32];
#pragma unroll
                        for (int k = 0; k < 32; ++k) v[k] = colv[2 * (i + k)];
#pragma unroll
                        for (int k = 0; k < 32; ++k) acc = __fadd_rn(acc, v[k]);
                    }
                } else {
                    for (; i + 32 <= cnt; i += 32) {
                        float v[32];
#pragma unroll
                        for (int k = 0; k < 32; ++k) v[k] = colv[2 * (i + k)];
#pragma unroll
                        for (int k = 0; k < 32; ++k) acc = __fadd_rn(acc, fabsf(__fsub_rn(v[k], mean)));
                    }
                }
                const float* col = reinterpret_cast<const float*>(s_kp[fr]) + ax;
                for (; i < cnt; ++i)
                    acc = pass == 0 ? __fadd_rn(acc, col[2 * i]) : __fadd_rn(acc, fabsf(__fsub_rn(col[2 * i], mean)));
            }
        }
        if (pass == 0) mean = __fdiv_rn(acc, (float)n);
        acc = pass == 0 ? 0.f : __fdiv_rn(acc, (float)n);
    }
    if (tid < 4) {
        s_mean[tid] = mean;
        s_scale[tid] = (float)(1.0 / (double)acc);  // float sX = 1.0/meanDevX
    }
    __syncthreads();
    // the normalised points: from the staged keypoints when each frame fit
    // one chunk (still in LDS), else re-read
    const bool staged = nmax <= kNormChunk;
    for (int i = tid; i < n1 + n2; i += kNormThreads) {
        const int fr = i >= n1, j = fr ? i - n1 : i;
        const float* k = fr ? kp2 : kp1;
        const float2 p = staged ? s_kp[fr][j] : make_float2(k[2 * j], k[2 * j + 1]);
        const float x = __fmul_rn(__fsub_rn(p.x, s_mean[2 * fr]), s_scale[2 * fr]);
        const float y = __fmul_rn(__fsub_rn(p.y, s_mean[2 * fr + 1]), s_scale[2 * fr + 1]);
        work[2 * i] = x;
        work[2 * i + 1] = y;
    }
    if (tid < 2) {  // T = [sX 0 -meanX*sX; 0 sY -meanY*sY; 0 0 1]
        float* T = work + 2 * (n1 + n2) + 9 * tid;
        const float sx = s_scale[2 * tid], sy = s_scale[2 * tid + 1];
        T[0] = sx; T[1] = 0.f; T[2] = __fmul_rn(-s_mean[2 * tid], sx);
        T[3] = 0.f; T[4] = sy; T[5] = __fmul_rn(-s_mean[2 * tid + 1], sy);
        T[6] = 0.f; T[7] = 0.f; T[8] = 1.f;
    }
    if (pts)
        for (int m = tid; m < nm; m += kNormThreads) {
            const int a = pairs[2 * m], b = pairs[2 * m + 1];
            const float2 p1 = staged ? s_kp[0][a] : make_float2(kp1[2 * a], kp1[2 * a + 1]);
            const float2 p2 = staged ? s_kp[1][b] : make_float2(kp2[2 * b], kp2[2 * b + 1]);
            pts[m] = make_float4(p1.x, p1.y, p2.x, p2.y);
        }
}

// float 3x3 product with double accumulation (OpenCV gemm on small float Mats)
__device__ void mul3(const float* a, const float* b, float* c) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = (float)((double)a[3 * i] * b[j] + (double)a[3 * i + 1] * b[3 + j] +
                                   (double)a[3 * i + 2] * b[6 + j]);
}

// cv::Mat::inv() of a 3x3 CV_32F (invert, DECOMP_LU, n == 3 closed form):
// det in double, cofactors in double times 1/det, rounded to float
__device__ void inv3(const float* m, float* o) {
    auto S = [&](int r, int c) { return (double)m[3 * r + c]; };
    const double d0 = S(0, 0) * (S(1, 1) * S(2, 2) - S(1, 2) * S(2, 1)) -
                      S(0, 1) * (S(1, 0) * S(2, 2) - S(1, 2) * S(2, 0)) +
                      S(0, 2) * (S(1, 0) * S(2, 1) - S(1, 1) * S(2, 0));
    if (d0 == 0.0) {
        for (int k = 0; k < 9; ++k) o[k] = 0.f;
        return;
    }
    const double d = 1.0 / d0;
    o[0] = (float)((S(1, 1) * S(2, 2) - S(1, 2) * S(2, 1)) * d);
    o[1] = (float)((S(0, 2) * S(2, 1) - S(0, 1) * S(2, 2)) * d);
    o[2] = (float)((S(0, 1) * S(1, 2) - S(0, 2) * S(1, 1)) * d);
    o[3] = (float)((S(1, 2) * S(2, 0) - S(1, 0) * S(2, 2)) * d);
    o[4] = (float)((S(0, 0) * S(2, 2) - S(0, 2) * S(2, 0)) * d);
    o[5] = (float)((S(0, 2) * S(1, 0) - S(0, 0) * S(1, 2)) * d);
    o[6] = (float)((S(1, 0) * S(2, 1) - S(1, 1) * S(2, 0)) * d);
    o[7] = (float)((S(0, 1) * S(2, 0) - S(0, 0) * S(2, 1)) * d);
    o[8] = (float)((S(0, 0) * S(1, 1) - S(0, 1) * S(1, 0)) * d);
}

constexpr int kModelThreads = 64;  // one wave per hypothesis

using ModelJacobi = orbgpu::JacobiLds<9, 16>;  // 9 columns, up to 16 rows (H: 16, F: 8 + zero rows)

__global__ __launch_bounds__(kModelThreads) void init_models_kernel(const float* __restrict__ work, int n1, int n2,
                                                                    const int* __restrict__ pairs,
                                                                    const int* __restrict__ sets, int n_iter,
                                                                    float* __restrict__ h21, float* __restrict__ h12,
                                                                    float* __restrict__ f21) {
    __shared__ double s_jac[ModelJacobi::kDoubles];
    const int lane = threadIdx.x;
    const int t = blockIdx.x;  // grid = 2 n_iter: H of every iteration, then F
    const bool valid = t < 2 * n_iter;
    const bool homography = t < n_iter;
    const int it = homography ? t : t - n_iter;
    const float* pn1 = work;
    const float* pn2 = work + 2 * n1;
    const float* T1 = work + 2 * (n1 + n2);
    const float* T2 = T1 + 9;
    double* A = s_jac;
    double* V = s_jac + ModelJacobi::M * ModelJacobi::NRP;
    double* nrm = V + ModelJacobi::M * ModelJacobi::NVP;
    ModelJacobi::init(A, V, lane, [](int, int) { return 0.0; });
    // lane r < 16 writes row r of A (float entries as the reference computes
    // them, held in double)
    if (valid && lane < 16) {
        const int r = lane;
        double a[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) a[k] = 0.0;
        const int i = homography ? (r >> 1) : r;  // the pair this row comes from
        if (i < 8) {
            const int idx = sets[8 * it + i];
            const int pa = pairs[2 * idx], pb = pairs[2 * idx + 1];
            const float u1 = pn1[2 * pa], v1 = pn1[2 * pa + 1], u2 = pn2[2 * pb], v2 = pn2[2 * pb + 1];
            if (homography) {
                if ((r & 1) == 0) {  // [0 0 0 -u1 -v1 -1 v2*u1 v2*v1 v2]
                    a[3] = -u1; a[4] = -v1; a[5] = -1.0;
                    a[6] = __fmul_rn(v2, u1); a[7] = __fmul_rn(v2, v1); a[8] = v2;
                } else {             // [u1 v1 1 0 0 0 -u2*u1 -u2*v1 -u2]
                    a[0] = u1; a[1] = v1; a[2] = 1.0;
                    a[6] = -__fmul_rn(u2, u1); a[7] = -__fmul_rn(u2, v1); a[8] = -u2;
                }
            } else {  // [u2*u1 u2*v1 u2 v2*u1 v2*v1 v2 u1 v1 1]
                a[0] = __fmul_rn(u2, u1); a[1] = __fmul_rn(u2, v1); a[2] = u2;
                a[3] = __fmul_rn(v2, u1); a[4] = __fmul_rn(v2, v1); a[5] = v2;
                a[6] = u1; a[7] = v1; a[8] = 1.0;
            }
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) A[k * ModelJacobi::NRP + r] = a[k];
    }
    ModelJacobi::sync();
    ModelJacobi::run(A, V, nrm, lane);
    // singular values = column norms; the first smallest decides vt.row(8)
    if (lane != 0 || !valid) return;
    int jmin = 0;
    double smin = 0.0;
    for (int j = 0; j < 9; ++j) {
        const double sj = sqrt(nrm[j]);
        if (j == 0 || sj < smin) {
            smin = sj;
            jmin = j;
        }
    }
    float nv[9];
    for (int k = 0; k < 9; ++k) nv[k] = (float)V[jmin * ModelJacobi::NVP + k];
    if (homography) {
        float T2inv[9], tmp[9], H[9], Hi[9];
        inv3(T2, T2inv);       // T2.inv()
        mul3(T2inv, nv, tmp);  // H21i = T2inv*Hn*T1
        mul3(tmp, T1, H);
        inv3(H, Hi);           // H12i = H21i.inv()
        for (int k = 0; k < 9; ++k) {
            h21[9 * it + k] = H[k];
            h12[9 * it + k] = Hi[k];
        }
    } else {
        // SVDecomp(Fpre): w(2) = 0; Fn = u*diag(w)*vt = sum of the two largest
        // singular triples
        double B[9], sv[3], V[9];
        for (int k = 0; k < 9; ++k) B[k] = nv[k];
        orbgpu::epnp::svd_hestenes<3, 3>(B, sv, V);
        int jm = 0;
        for (int j = 1; j < 3; ++j)
            if (sv[j] < sv[jm]) jm = j;
        float Fn[9];
        for (int rr = 0; rr < 3; ++rr)
            for (int cc = 0; cc < 3; ++cc) {
                double acc = 0.0;
                for (int j = 0; j < 3; ++j)
                    if (j != jm) acc += B[3 * rr + j] * V[3 * cc + j];  // (U_j s_j) v_j^T
                Fn[3 * rr + cc] = (float)acc;
            }
        float T2t[9], tmp[9], F[9];
        for (int rr = 0; rr < 3; ++rr)
            for (int cc = 0; cc < 3; ++cc) T2t[3 * rr + cc] = T2[3 * cc + rr];
        mul3(T2t, Fn, tmp);  // F21i = T2t*Fn*T1
        mul3(tmp, T1, F);
        for (int k = 0; k < 9; ++k) f21[9 * it + k] = F[k];
    }
}

}  // namespace

extern "C" size_t orbgpu_init_workspace_bytes(int n1, int n2) {
    return (size_t)(2 * ((n1 > 0 ? n1 : 0) + (n2 > 0 ? n2 : 0)) + 18) * sizeof(float);
}

extern "C" int orbgpu_init_hypotheses_batch_device(const float* d_kp1, int n1, const float* d_kp2, int n2,
                                                   const int* d_pairs, int n_matches, const int* d_sets, int n_iter,
                                                   void* d_work, orbgpu_match_pts* d_pts, float* d_h21,
                                                   float* d_h12, float* d_f21, void* stream) {
    if (n1 <= 0 || n2 <= 0 || n_matches < 8 || n_iter < 0 || !d_kp1 || !d_kp2 || !d_pairs || !d_work ||
        (n_iter > 0 && (!d_sets || !d_h21 || !d_h12 || !d_f21)))
        return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument (needs >= 8 matches and keypoints in both frames)");
    if ((uintptr_t)d_pts & 15) return orbgpu::fail(ORBGPU_ERR_ARG, "d_pts must be 16-byte aligned");
    if (((uintptr_t)d_kp1 | (uintptr_t)d_kp2) & 7)
        return orbgpu::fail(ORBGPU_ERR_ARG, "d_kp1 / d_kp2 must be 8-byte aligned (x, y float pairs)");
    if (int rc = orbgpu::check_device()) return rc;
    (void)hipGetLastError();
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(init_normalize_kernel, dim3(1), dim3(kNormThreads), 0, s, d_kp1, n1, d_kp2, n2, d_pairs,
                       n_matches, static_cast<float*>(d_work), reinterpret_cast<float4*>(d_pts));
    ORB_HIP(hipGetLastError());
    if (n_iter > 0) {
        hipLaunchKernelGGL(init_models_kernel, dim3(2 * n_iter), dim3(kModelThreads), 0, s, static_cast<const float*>(d_work), n1, n2, d_pairs, d_sets,
                           n_iter, d_h21, d_h12, d_f21);
        ORB_HIP(hipGetLastError());
    }
    return ORBGPU_OK;
}
