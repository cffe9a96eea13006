// init.hip -- Initializer::CheckHomography (Initializer.cpp:390-495) and
// CheckFundamental (:497-594) for a batch of RANSAC hypotheses over the same
// matches (include/orbgpu_init.h).
//
// One 256-thread workgroup per hypothesis; the matches are walked in chunks
// of 4096, lanes striding over the chunk.  Each lane evaluates both transfer errors exactly
// as the reference writes them (-ffp-contract=off, the reciprocal 1.0/w in
// double as the reference's double literal makes it) and writes its inlier
// byte (coalesced).  The two score terms of every match of the chunk go to LDS and lane 0
// adds them in match order, so the float score is the reference loop's sum
// bit for bit.  A term the reference skips (chi-square above threshold) is
// stored as +0, which leaves a score that is never -0 unchanged; a NaN
// chi-square is not above threshold, so its NaN term propagates as there.
// The per-match work is a few dozen flops on 16 bytes: the launch is latency
// bound (one dependent add chain of 2n per workgroup), not HBM bound.
#include <hip/hip_runtime.h>

#include "../../include/orbgpu_init.h"
#include "host_common.h"

namespace {

constexpr int kInitThreads = 256;
constexpr int kInitChunk = 4096;  // matches staged per pass: 32 KiB of terms in LDS

__device__ __forceinline__ float recip_d(float w) { return (float)(1.0 / (double)w); }

// the staged score terms -> the running score, in match order (lane 0).
// Eight 16-byte LDS reads are issued together ahead of their 32 dependent
// adds, so the chain waits on LDS once per 16 matches, not once per 2.
__device__ __forceinline__ float add_terms(const float* s_t, int cnt, float score) {
    const float4* s4 = reinterpret_cast<const float4*>(s_t);
    int i = 0;
    for (; i + 16 <= cnt; i += 16) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = s4[(i >> 1) + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            score += v[k].x;
            score += v[k].y;
            score += v[k].z;
            score += v[k].w;
        }
    }
    for (; i < cnt; ++i) {
        score += s_t[2 * i];
        score += s_t[2 * i + 1];
    }
    return score;
}

template <bool kHomography>
__device__ __forceinline__ void check_body(int h, float* s_t, const float4* __restrict__ pts, int n,
                                           const float* __restrict__ ma, const float* __restrict__ mb,
                                           float inv_sigma2, float* __restrict__ scores,
                                           uint8_t* __restrict__ inliers) {
    const int tid = threadIdx.x;
    float a[9], b[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = ma[9 * h + k];
    if (kHomography) {
#pragma unroll
        for (int k = 0; k < 9; ++k) b[k] = mb[9 * h + k];
    }
    uint8_t* inl = inliers + (size_t)h * (size_t)n;
    float score = 0.f;
    for (int base = 0; base < n; base += kInitChunk) {
        const int cnt = min(kInitChunk, n - base);
        for (int j = tid; j < cnt; j += kInitThreads) {
            const int i = base + j;
            const float4 p = pts[i];
            const float u1 = p.x, v1 = p.y, u2 = p.z, v2 = p.w;
            float chi1, chi2, th, ths;
            if (kHomography) {
                th = (float)5.991;
                ths = th;
                // H12 maps image 2 into image 1 (:435-442)
                const float w2in1inv = recip_d(b[6] * u2 + b[7] * v2 + b[8]);
                const float u2in1 = (b[0] * u2 + b[1] * v2 + b[2]) * w2in1inv;
                const float v2in1 = (b[3] * u2 + b[4] * v2 + b[5]) * w2in1inv;
                const float d1 = (u1 - u2in1) * (u1 - u2in1) + (v1 - v2in1) * (v1 - v2in1);
                chi1 = d1 * inv_sigma2;
                // H21 maps image 1 into image 2 (:458-465)
                const float w1in2inv = recip_d(a[6] * u1 + a[7] * v1 + a[8]);
                const float u1in2 = (a[0] * u1 + a[1] * v1 + a[2]) * w1in2inv;
                const float v1in2 = (a[3] * u1 + a[4] * v1 + a[5]) * w1in2inv;
                const float d2 = (u2 - u1in2) * (u2 - u1in2) + (v2 - v1in2) * (v2 - v1in2);
                chi2 = d2 * inv_sigma2;
            } else {
                th = (float)3.841;
                ths = (float)5.991;
                // epipolar line of x1 in image 2 (:542-551)
                const float a2 = a[0] * u1 + a[1] * v1 + a[2];
                const float b2 = a[3] * u1 + a[4] * v1 + a[5];
                const float c2 = a[6] * u1 + a[7] * v1 + a[8];
                const float num2 = a2 * u2 + b2 * v2 + c2;
                chi1 = (num2 * num2 / (a2 * a2 + b2 * b2)) * inv_sigma2;
                // epipolar line of x2 in image 1 (:562-571)
                const float a1 = a[0] * u2 + a[3] * v2 + a[6];
                const float b1 = a[1] * u2 + a[4] * v2 + a[7];
                const float c1 = a[2] * u2 + a[5] * v2 + a[8];
                const float num1 = a1 * u1 + b1 * v1 + c1;
                chi2 = (num1 * num1 / (a1 * a1 + b1 * b1)) * inv_sigma2;
            }
            const bool out1 = chi1 > th, out2 = chi2 > th;
            s_t[2 * j] = out1 ? 0.f : ths - chi1;
            s_t[2 * j + 1] = out2 ? 0.f : ths - chi2;
            inl[i] = (uint8_t)!(out1 || out2);
        }
        __syncthreads();
        if (tid == 0) score = add_terms(s_t, cnt, score);
        __syncthreads();
    }
    if (tid == 0) scores[h] = score;
}

template <bool kHomography>
__global__ __launch_bounds__(kInitThreads) void init_check_kernel(const float4* __restrict__ pts, int n,
                                                                  const float* __restrict__ ma,
                                                                  const float* __restrict__ mb, float inv_sigma2,
                                                                  float* __restrict__ scores,
                                                                  uint8_t* __restrict__ inliers) {
    __shared__ __attribute__((aligned(16))) float s_t[2 * kInitChunk];
    check_body<kHomography>(blockIdx.x, s_t, pts, n, ma, mb, inv_sigma2, scores, inliers);
}

// both models in one grid -- the reference runs FindHomography and
// FindFundamental concurrently in two threads (Initializer.cpp:133-138)
__global__ __launch_bounds__(kInitThreads) void init_check_both_kernel(
    const float4* __restrict__ pts, int n, const float* __restrict__ h21, const float* __restrict__ h12, int nh,
    const float* __restrict__ f21, float inv_sigma2, float* __restrict__ scores_h, uint8_t* __restrict__ inl_h,
    float* __restrict__ scores_f, uint8_t* __restrict__ inl_f) {
    __shared__ __attribute__((aligned(16))) float s_t[2 * kInitChunk];
    const int b = blockIdx.x;
    if (b < nh)
        check_body<true>(b, s_t, pts, n, h21, h12, inv_sigma2, scores_h, inl_h);
    else
        check_body<false>(b - nh, s_t, pts, n, f21, f21, inv_sigma2, scores_f, inl_f);
}

int launch(bool homography, const orbgpu_match_pts* d_pts, int n, const float* d_a, const float* d_b, int nhyp,
           float sigma, float* d_scores, uint8_t* d_inliers, void* stream) {
    if ((n > 0 && !d_pts) || !d_a || (homography && !d_b) || !d_scores || (n > 0 && !d_inliers) || n < 0 || nhyp < 0 ||
        !(sigma > 0.f))
        return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    if ((uintptr_t)d_pts & 15) return orbgpu::fail(ORBGPU_ERR_ARG, "d_pts must be 16-byte aligned (float4 loads)");
    if (nhyp == 0) return ORBGPU_OK;
    if (int rc = orbgpu::check_device()) return rc;
    (void)hipGetLastError();
    // invSigmaSquare = 1.0/(sigma*sigma) (:411, :516)
    const float inv_sigma2 = (float)(1.0 / (double)(sigma * sigma));
    const float4* pts = reinterpret_cast<const float4*>(d_pts);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (homography)
        hipLaunchKernelGGL(init_check_kernel<true>, dim3(nhyp), dim3(kInitThreads), 0, s, pts, n, d_a, d_b,
                           inv_sigma2, d_scores, d_inliers);
    else
        hipLaunchKernelGGL(init_check_kernel<false>, dim3(nhyp), dim3(kInitThreads), 0, s, pts, n, d_a, d_a,
                           inv_sigma2, d_scores, d_inliers);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

}  // namespace

extern "C" int orbgpu_init_check_homography_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_h21,
                                                         const float* d_h12, int nhyp, float sigma, float* d_scores,
                                                         uint8_t* d_inliers, void* stream) {
    return launch(true, d_pts, n, d_h21, d_h12, nhyp, sigma, d_scores, d_inliers, stream);
}

extern "C" int orbgpu_init_check_fundamental_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_f21,
                                                          int nhyp, float sigma, float* d_scores, uint8_t* d_inliers,
                                                          void* stream) {
    return launch(false, d_pts, n, d_f21, nullptr, nhyp, sigma, d_scores, d_inliers, stream);
}

extern "C" int orbgpu_init_check_both_batch_device(const orbgpu_match_pts* d_pts, int n, const float* d_h21,
                                                   const float* d_h12, int nh, const float* d_f21, int nf,
                                                   float sigma, float* d_scores_h, uint8_t* d_inliers_h,
                                                   float* d_scores_f, uint8_t* d_inliers_f, void* stream) {
    if ((n > 0 && !d_pts) || n < 0 || nh < 0 || nf < 0 || !(sigma > 0.f) ||
        (nh > 0 && (!d_h21 || !d_h12 || !d_scores_h || (n > 0 && !d_inliers_h))) ||
        (nf > 0 && (!d_f21 || !d_scores_f || (n > 0 && !d_inliers_f))))
        return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    if ((uintptr_t)d_pts & 15) return orbgpu::fail(ORBGPU_ERR_ARG, "d_pts must be 16-byte aligned (float4 loads)");
    if (nh + nf == 0) return ORBGPU_OK;
    if (int rc = orbgpu::check_device()) return rc;
    (void)hipGetLastError();
    const float inv_sigma2 = (float)(1.0 / (double)(sigma * sigma));
    hipLaunchKernelGGL(init_check_both_kernel, dim3(nh + nf), dim3(kInitThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float4*>(d_pts), n, d_h21,
                       d_h12, nh, d_f21, inv_sigma2, d_scores_h, d_inliers_h, d_scores_f, d_inliers_f);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

extern "C" int orbgpu_init_select_best(const float* scores, int nhyp, int* best_out) {
    if ((!scores && nhyp > 0) || nhyp < 0 || !best_out) return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    float best = 0.f;
    int idx = -1;
    for (int h = 0; h < nhyp; ++h)
        if (scores[h] > best) {
            best = scores[h];
            idx = h;
        }
    *best_out = idx;
    return ORBGPU_OK;
}
