// init_reconstruct.hip -- Initializer::ReconstructH / ReconstructF
// (src/Initializer.cpp:596-963) with CheckRT (:1017-1118), Triangulate
// (:930-945) and DecomposeE (:1120-1150) (include/orbgpu_init.h,
// orbgpu_init_reconstruct).
//
// The motion hypotheses are a handful of 3x3 decompositions per call and
// are built on the host (8 for a homography, 4 for an essential matrix);
// CheckRT -- a 4x4 linear triangulation plus the depth, parallax and
// reprojection tests for every inlier match under every hypothesis -- is
// the data-parallel part and runs on the GPU: one thread per (match,
// hypothesis) over the whole chip (check_rt_kernel), then one block per
// hypothesis counts nGood and finds the parallax the reference reads after
// sorting (the min(50, nGood-1)-th smallest cosine) by a radix select
// (rt_parallax_kernel).  (Round 2 ran one block per hypothesis with an
// order-statistic walk: 177 us for 8 hypotheses x 1000 matches.)
//
// OpenCV's SVDs (cv::SVD::compute of float Mats, Jacobi in float) are not
// reproducible bit for bit: the 3x3 decompositions and each match's 4x4
// null vector are computed by one-sided Jacobi in double and rounded to
// float where the reference holds floats.  Every other operation follows
// the reference's float expression order.  Sign conventions of the SVD only
// reorder the hypothesis set, the kept motion is the
// same.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/orbgpu_init.h"
#include "epnp.h"
#include "host_common.h"
#include "host_ctx.h"
#include "group_sum.h"

namespace orbgpu {

namespace {

constexpr int kRecThreads = 256;
constexpr int kRecMaxMatches = 16384;  // LDS: one u32 cosine key per match

struct RecHyp {
    float R[9], t[3];
    float P2[12];  // K*[R|t]
    float O2[3];   // -R^T t
};

__device__ inline float dotd3f(const float* a, const float* x) {  // cv::Mat product, double accumulation
    return (float)((double)a[0] * x[0] + (double)a[1] * x[1] + (double)a[2] * x[2]);
}

// float -> u32 key with the float order (no NaN expected)
__device__ inline unsigned ord_key(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float key_float(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__global__ __launch_bounds__(kRecThreads) void check_rt_kernel(const float4* __restrict__ pts,
                                                               const unsigned char* __restrict__ inl, int n,
                                                               const RecHyp* __restrict__ hyps, float fx, float fy,
                                                               float cx, float cy, float th2,
                                                               unsigned char* __restrict__ good,
                                                               float* __restrict__ p3d,
                                                               unsigned* __restrict__ keys) {
    const int h = blockIdx.y, m = blockIdx.x * kRecThreads + threadIdx.x;
    const RecHyp H = hyps[h];
    if (m < n) {
        unsigned key = ~0u;
        unsigned char gflag = 0;
        float X[3] = {0.f, 0.f, 0.f};
        if (inl[m]) {
            const float4 p = pts[m];  // (kp1.x, kp1.y, kp2.x, kp2.y)
            // Triangulate (:930-945): A rows = x * P.row(2) - P.row(0), ...; P1 = [K|0]
            double A[16];
            const float P1r0[4] = {fx, 0.f, cx, 0.f}, P1r1[4] = {0.f, fy, cy, 0.f}, P1r2[4] = {0.f, 0.f, 1.f, 0.f};
            for (int c = 0; c < 4; ++c) {
                A[c] = (double)(p.x * P1r2[c] - P1r0[c]);
                A[4 + c] = (double)(p.y * P1r2[c] - P1r1[c]);
                A[8 + c] = (double)(p.z * H.P2[8 + c] - H.P2[c]);
                A[12 + c] = (double)(p.w * H.P2[8 + c] - H.P2[4 + c]);
            }
            double s[4], v[16];
            epnp::svd_hestenes<4, 4>(A, s, v);
            int jmin = 0;
            for (int j = 1; j < 4; ++j)
                if (s[j] < s[jmin]) jmin = j;
            const float w3 = (float)v[12 + jmin];  // x3D = vt.row(3).t(); rowRange(0,3) / x3D(3)
            for (int k = 0; k < 3; ++k) X[k] = (float)v[4 * k + jmin] / w3;
            bool ok = isfinite(X[0]) && isfinite(X[1]) && isfinite(X[2]);
            float cosPar = 0.f;
            if (ok) {
                const float dist1 = (float)sqrt((double)X[0] * X[0] + (double)X[1] * X[1] + (double)X[2] * X[2]);
                const float n2[3] = {X[0] - H.O2[0], X[1] - H.O2[1], X[2] - H.O2[2]};
                const float dist2 = (float)sqrt((double)n2[0] * n2[0] + (double)n2[1] * n2[1] + (double)n2[2] * n2[2]);
                const double dot = (double)X[0] * n2[0] + (double)X[1] * n2[1] + (double)X[2] * n2[2];
                cosPar = (float)(dot / (double)(dist1 * dist2));
                if (X[2] <= 0.f && (double)cosPar < 0.99998) ok = false;
                float Xc2[3];
                for (int r = 0; r < 3; ++r) Xc2[r] = dotd3f(H.R + 3 * r, X) + H.t[r];
                if (ok && Xc2[2] <= 0.f && (double)cosPar < 0.99998) ok = false;
                if (ok) {
                    const float invZ1 = 1.0f / X[2];
                    const float im1x = fx * X[0] * invZ1 + cx, im1y = fy * X[1] * invZ1 + cy;
                    const float e1 = (im1x - p.x) * (im1x - p.x) + (im1y - p.y) * (im1y - p.y);
                    if (e1 > th2) ok = false;
                }
                if (ok) {
                    const float invZ2 = 1.0f / Xc2[2];
                    const float im2x = fx * Xc2[0] * invZ2 + cx, im2y = fy * Xc2[1] * invZ2 + cy;
                    const float e2 = (im2x - p.z) * (im2x - p.z) + (im2y - p.w) * (im2y - p.w);
                    if (e2 > th2) ok = false;
                }
            }
            if (ok) {
                key = min(ord_key(cosPar), 0xFFFFFFFEu);  // ~0u marks a match CheckRT did not count
                gflag = (double)cosPar < 0.99998 ? 1 : 0;
            } else {
                X[0] = X[1] = X[2] = 0.f;
            }
        }
        keys[(size_t)h * n + m] = key;
        good[(size_t)h * n + m] = key != ~0u ? (unsigned char)(gflag | 2) : 0;  // bit 1: counted in nGood
        float* o = p3d + 3 * ((size_t)h * n + m);
        o[0] = X[0];
        o[1] = X[1];
        o[2] = X[2];
    }
}

// nGood and the parallax of one hypothesis (:1102-1110): the count of the
// counted matches and the k-th smallest of their cosines, k = min(50,
// nGood - 1) -- vCosParallax[k] after the reference's sort -- by a radix
// select (four 8-bit histogram passes in LDS) over the keys check_rt_kernel
// wrote; matches it did not count carry ~0u, above every counted key, so they
// never reach rank k < nGood
constexpr int kSelThreads = 1024;
__global__ __launch_bounds__(kSelThreads) void rt_parallax_kernel(const unsigned* __restrict__ keys, int n,
                                                                  int* __restrict__ n_good,
                                                                  float* __restrict__ parallax) {
    __shared__ int s_hist[256];
    __shared__ int s_wsum[kSelThreads / 64];
    __shared__ unsigned s_prefix;
    __shared__ int s_k;
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned* K = keys + (size_t)h * n;
    int cnt = 0;
    for (int m = tid; m < n; m += kSelThreads) cnt += K[m] != ~0u;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) s_wsum[wave] = cnt;
    __syncthreads();
    int ng = 0;
    for (int w = 0; w < kSelThreads / 64; ++w) ng += s_wsum[w];
    if (ng == 0) {
        if (tid == 0) {
            n_good[h] = 0;
            parallax[h] = 0.f;
        }
        return;
    }
    if (tid == 0) {
        s_prefix = 0u;
        s_k = min(50, ng - 1);
    }
    unsigned mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) s_hist[tid] = 0;
        __syncthreads();
        const unsigned prefix = s_prefix;
        for (int m = tid; m < n; m += kSelThreads) {
            const unsigned key = K[m];
            if ((key & mask) == prefix) atomicAdd(&s_hist[(key >> shift) & 255u], 1);
        }
        __syncthreads();
        if (wave == 0) {  // the bin holding rank k: lane owns bins 4 lane .. 4 lane + 3
            int c[4], sum = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = s_hist[4 * lane + q];
                sum += c[q];
            }
            const int incl = wave_incl_scan_dpp(sum);
            const int k = s_k;
            int below = incl - sum;
            if (below <= k && k < incl) {  // exactly one lane
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (k < below + c[q]) {
                        s_prefix = prefix | ((unsigned)(4 * lane + q) << shift);
                        s_k = k - below;
                        break;
                    }
                    below += c[q];
                }
            }
        }
        mask |= 255u << shift;
        __syncthreads();
    }
    if (tid == 0) {
        // parallax = acos(c) * 180 / CV_PI (float acos, float * int, then the double division)
        n_good[h] = ng;
        parallax[h] = (float)((double)(acosf(key_float(s_prefix)) * 180) / 3.14159265358979323846);
    }
}

// ---- host: the 3x3 decompositions ------------------------------------------------
void mul3h(const float* a, const float* b, float* c) {  // float gemm, double accumulation
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = (float)((double)a[3 * i] * b[j] + (double)a[3 * i + 1] * b[3 + j] +
                                   (double)a[3 * i + 2] * b[6 + j]);
}

void inv3h(const float* m, float* o) {  // cv::Mat::inv() of a 3x3 CV_32F (closed form, double)
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

double det3(const float* m) {  // cv::determinant of a 3x3 CV_32F (double)
    auto S = [&](int r, int c) { return (double)m[3 * r + c]; };
    return S(0, 0) * (S(1, 1) * S(2, 2) - S(1, 2) * S(2, 1)) - S(0, 1) * (S(1, 0) * S(2, 2) - S(1, 2) * S(2, 0)) +
           S(0, 2) * (S(1, 0) * S(2, 1) - S(1, 1) * S(2, 0));
}

// cv::SVD::compute of a 3x3 float matrix: w descending, U and Vt as floats.
// Jacobi on the columns in double; U's third column completes a right-handed
// basis when sigma3 is ~0 (E: rank 2), any consistent choice only reorders
// the reference's hypothesis set.
void svd3(const float* M, float* w, float* U, float* Vt) {
    double a[9], s[3], v[9];
    for (int k = 0; k < 9; ++k) a[k] = M[k];
    epnp::svd_hestenes<3, 3>(a, s, v);
    int o[3] = {0, 1, 2};
    std::sort(o, o + 3, [&](int x, int y) { return s[x] > s[y]; });
    double u[3][3], vv[3][3];
    for (int j = 0; j < 3; ++j) {
        for (int k = 0; k < 3; ++k) vv[j][k] = v[3 * k + o[j]];
        for (int k = 0; k < 3; ++k) u[j][k] = s[o[j]] > 0 ? a[3 * k + o[j]] / s[o[j]] : 0.0;
    }
    if (!(s[o[2]] > 1e-9 * s[o[0]])) {  // u3 = u1 x u2
        u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
        u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
        u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    }
    for (int j = 0; j < 3; ++j) {
        w[j] = (float)s[o[j]];
        for (int k = 0; k < 3; ++k) {
            U[3 * k + j] = (float)u[j][k];
            Vt[3 * j + k] = (float)vv[j][k];
        }
    }
}

void scale_norm(float* t) {  // t = t / cv::norm(t): double norm, alpha = 1/norm
    const double nrm = std::sqrt((double)t[0] * t[0] + (double)t[1] * t[1] + (double)t[2] * t[2]);
    const double al = 1.0 / nrm;
    for (int k = 0; k < 3; ++k) t[k] = (float)((double)t[k] * al);
}

// ReconstructH's eight (R, t) (:707-850); false when d1/d2 or d2/d3 < 1.00001
bool homography_hyps(const float* H21, const float* K, std::vector<RecHyp>& hy) {
    float invK[9], tmp[9], A[9], U[9], w[3], Vt[9];
    inv3h(K, invK);
    mul3h(invK, H21, tmp);
    mul3h(tmp, K, A);
    svd3(A, w, U, Vt);
    const float s = (float)(det3(U) * det3(Vt));
    const float d1 = w[0], d2 = w[1], d3 = w[2];
    if ((double)(d1 / d2) < 1.00001 || (double)(d2 / d3) < 1.00001) return false;
    const float aux1 = std::sqrt((d1 * d1 - d2 * d2) / (d1 * d1 - d3 * d3));
    const float aux3 = std::sqrt((d2 * d2 - d3 * d3) / (d1 * d1 - d3 * d3));
    const float x1[4] = {aux1, aux1, -aux1, -aux1}, x3[4] = {aux3, -aux3, aux3, -aux3};
    const float aux_st = std::sqrt((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 + d3) * d2);
    const float cth = (d2 * d2 + d1 * d3) / ((d1 + d3) * d2);
    const float st[4] = {aux_st, -aux_st, -aux_st, aux_st};
    const float aux_sp = std::sqrt((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 - d3) * d2);
    const float cph = (d1 * d3 - d2 * d2) / ((d1 - d3) * d2);
    const float sp[4] = {aux_sp, -aux_sp, -aux_sp, aux_sp};
    for (int pass = 0; pass < 2; ++pass)
        for (int i = 0; i < 4; ++i) {
            float Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            float tp[3];
            if (pass == 0) {  // d' = d2 (:734-782)
                Rp[0] = cth; Rp[2] = -st[i]; Rp[6] = st[i]; Rp[8] = cth;
                tp[0] = x1[i]; tp[1] = 0; tp[2] = -x3[i];
                for (float& x : tp) x *= d1 - d3;
            } else {  // d' = -d2 (:786-836)
                Rp[0] = cph; Rp[2] = sp[i]; Rp[4] = -1; Rp[6] = sp[i]; Rp[8] = -cph;
                tp[0] = x1[i]; tp[1] = 0; tp[2] = x3[i];
                for (float& x : tp) x *= d1 + d3;
            }
            RecHyp hh{};
            float sU[9], URp[9];
            for (int r = 0; r < 3; ++r)  // s*U*Rp: one gemm with alpha = s
                for (int c = 0; c < 3; ++c)
                    URp[3 * r + c] = (float)(((double)U[3 * r] * Rp[c] + (double)U[3 * r + 1] * Rp[3 + c] +
                                              (double)U[3 * r + 2] * Rp[6 + c]) * (double)s);
            (void)sU;
            mul3h(URp, Vt, hh.R);
            for (int r = 0; r < 3; ++r)
                hh.t[r] = (float)((double)U[3 * r] * tp[0] + (double)U[3 * r + 1] * tp[1] + (double)U[3 * r + 2] * tp[2]);
            scale_norm(hh.t);
            hy.push_back(hh);
        }
    return true;
}

// DecomposeE (:1120-1150) and ReconstructF's four (R, t) in its order:
// (R1, t), (R2, t), (R1, -t), (R2, -t)
void fundamental_hyps(const float* F21, const float* K, std::vector<RecHyp>& hy) {
    float Kt[9], tmp[9], E[9], U[9], w[3], Vt[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Kt[3 * r + c] = K[3 * c + r];
    mul3h(Kt, F21, tmp);
    mul3h(tmp, K, E);
    svd3(E, w, U, Vt);
    float t[3] = {U[2], U[5], U[8]};
    scale_norm(t);
    const float W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1}, Wt[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    float uw[9], R1[9], R2[9];
    mul3h(U, W, uw);
    mul3h(uw, Vt, R1);
    if (det3(R1) < 0)
        for (float& x : R1) x = -x;
    mul3h(U, Wt, uw);
    mul3h(uw, Vt, R2);
    if (det3(R2) < 0)
        for (float& x : R2) x = -x;
    const float* Rs[4] = {R1, R2, R1, R2};
    for (int i = 0; i < 4; ++i) {
        RecHyp hh{};
        std::memcpy(hh.R, Rs[i], sizeof(hh.R));
        for (int k = 0; k < 3; ++k) hh.t[k] = i < 2 ? t[k] : -t[k];
        hy.push_back(hh);
    }
}

// FindHomography / FindFundamental's choice of the kept iteration for both
// models (`if (currentScore > score)` from score = 0: the first maximum among
// scores > 0, NaN never kept; Initializer.cpp:160-269), then the kept models
// and their inlier flags packed for ONE read-back: out = {bh, bf, SH bits, SF
// bits, H21[9], F21[9], inliersH[N], inliersF[N]} (zeros for -1).
struct PickKey {
    float v;
    int i;
};
__device__ inline PickKey pick_better(PickKey a, PickKey b) {
    return (b.v > a.v || (b.v == a.v && b.i >= 0 && (a.i < 0 || b.i < a.i))) ? b : a;
}
__global__ __launch_bounds__(256) void init_pick_kernel(const float* __restrict__ sh, const float* __restrict__ sf,
                                                        int it, const float* __restrict__ h21,
                                                        const float* __restrict__ f21, const uint8_t* __restrict__ ih,
                                                        const uint8_t* __restrict__ iff, int N,
                                                        uint8_t* __restrict__ out) {
    __shared__ PickKey s_k[2][4];
    __shared__ int s_best[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int m = 0; m < 2; ++m) {
        const float* sc = m ? sf : sh;
        PickKey k{0.f, -1};
        for (int h = tid; h < it; h += 256) {
            const float v = sc[h];
            if (v > k.v) k = PickKey{v, h};  // strided ascending: the thread's first maximum
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const PickKey q{__shfl_xor(k.v, o, 64), __shfl_xor(k.i, o, 64)};
            k = pick_better(k, q);
        }
        if (lane == 0) s_k[m][wave] = k;
    }
    __syncthreads();
    if (tid < 2) {
        PickKey k = s_k[tid][0];
        for (int w = 1; w < 4; ++w) k = pick_better(k, s_k[tid][w]);
        s_best[tid] = k.i;
        int* hdr = reinterpret_cast<int*>(out);
        hdr[tid] = k.i;
        hdr[2 + tid] = __float_as_int(k.i >= 0 ? k.v : 0.f);
    }
    __syncthreads();
    const int bh = s_best[0], bf = s_best[1];
    float* mo = reinterpret_cast<float*>(out + 16);
    if (tid < 18) {
        const int m = tid / 9, k = tid - 9 * m, b = m ? bf : bh;
        mo[tid] = b >= 0 ? (m ? f21 : h21)[9 * (size_t)b + k] : 0.f;
    }
    uint8_t* fl = out + 16 + 72;
    for (int i = tid; i < 2 * N; i += 256) {
        const int m = i >= N, j = m ? i - N : i, b = m ? bf : bh;
        fl[i] = b >= 0 ? (m ? iff : ih)[(size_t)b * N + j] : 0;
    }
}

}  // namespace

}  // namespace orbgpu

using namespace orbgpu;

extern "C" int orbgpu_init_reconstruct(int model, const float* kp1, int n1, const float* kp2, int n2,
                                       const int* pairs, int n_matches, const unsigned char* inliers,
                                       const float* M21, const float* K, float sigma, float min_parallax,
                                       int min_triangulated, orbgpu_init_reconstruction* out, float* p3d,
                                       unsigned char* triangulated) {
    if (!out || (model != ORBGPU_INIT_MODEL_H && model != ORBGPU_INIT_MODEL_F) || n1 < 0 || n2 < 0 ||
        n_matches < 0 || !M21 || !K || (n_matches > 0 && (!pairs || !inliers || !kp1 || !kp2)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (n_matches > kRecMaxMatches) return fail(ORBGPU_ERR_CAPACITY, "more than 16384 matches");
    for (int i = 0; i < n_matches; ++i)
        if (pairs[2 * i] < 0 || pairs[2 * i] >= n1 || pairs[2 * i + 1] < 0 || pairs[2 * i + 1] >= n2)
            return fail(ORBGPU_ERR_ARG, "match index out of range");
    std::memset(out, 0, sizeof(*out));
    out->best = -1;
    if (p3d) std::memset(p3d, 0, sizeof(float) * 3 * (size_t)n1);
    if (triangulated) std::memset(triangulated, 0, (size_t)n1);
    int N = 0;
    for (int i = 0; i < n_matches; ++i) N += inliers[i] ? 1 : 0;
    std::vector<RecHyp> hy;
    if (model == ORBGPU_INIT_MODEL_H) {
        if (!homography_hyps(M21, K, hy)) return ORBGPU_OK;  // ok = 0 (:703-706)
    } else {
        fundamental_hyps(M21, K, hy);
    }
    const int nh = (int)hy.size();
    out->n_hyp = nh;
    const float fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    for (RecHyp& h : hy) {  // P2 = K*[R|t] (:1042-1045), O2 = -R^T t (:1047)
        float Rt[12];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) Rt[4 * r + c] = h.R[3 * r + c];
            Rt[4 * r + 3] = h.t[r];
        }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c)
                h.P2[4 * r + c] = (float)((double)K[3 * r] * Rt[c] + (double)K[3 * r + 1] * Rt[4 + c] +
                                          (double)K[3 * r + 2] * Rt[8 + c]);
        for (int j = 0; j < 3; ++j)
            h.O2[j] = -(float)((double)h.R[j] * h.t[0] + (double)h.R[3 + j] * h.t[1] + (double)h.R[6 + j] * h.t[2]);
    }
    int rc = check_device();
    if (rc) return rc;
    const int n = std::max(n_matches, 1);
    std::vector<float> pts(4 * (size_t)n, 0.f);
    for (int i = 0; i < n_matches; ++i) {
        const int a = pairs[2 * i], b = pairs[2 * i + 1];
        pts[4 * i] = kp1[2 * a];
        pts[4 * i + 1] = kp1[2 * a + 1];
        pts[4 * i + 2] = kp2[2 * b];
        pts[4 * i + 3] = kp2[2 * b + 1];
    }
    std::vector<unsigned char> inl(n, 0);
    if (n_matches) std::memcpy(inl.data(), inliers, n_matches);
    const float mSigma2 = sigma * sigma;
    const float th2 = (float)(4.0 * mSigma2);
    const size_t nhn = (size_t)nh * n;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const float4* d_pts;
    const unsigned char* d_inl;
    const RecHyp* d_h;
    int* d_ng;
    float *d_par, *d_p3;
    unsigned char* d_good;
    unsigned* d_key;
    rc = call.run([&](HostCall& A) {
        d_pts = reinterpret_cast<const float4*>(A.in(pts.data(), pts.size()));
        d_inl = A.in(inl.data(), (size_t)n);
        d_h = A.in(hy.data(), (size_t)nh);
        d_ng = A.out<int>((size_t)nh);
        d_par = A.out<float>((size_t)nh);
        d_good = A.out<unsigned char>(nhn);
        d_p3 = A.out<float>(3 * nhn);
        d_key = A.out<unsigned>(nhn);  // scratch: the cosine keys between the two kernels
    });
    if (rc) return rc;
    std::vector<int> ng(nh);
    std::vector<float> par(nh);
    std::vector<unsigned char> good(nhn);
    std::vector<float> P3(3 * nhn);
    // one match per thread over every (match block, hypothesis): a few
    // hypotheses x ~1000 matches is far below one wave per SIMD otherwise
    if (n_matches > 0) {
        hipLaunchKernelGGL(check_rt_kernel, dim3((n_matches + kRecThreads - 1) / kRecThreads, nh), dim3(kRecThreads),
                           0, ctx->stream, d_pts, d_inl, n_matches, d_h, fx, fy, cx, cy, th2, d_good, d_p3, d_key);
        ORB_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(rt_parallax_kernel, dim3(nh), dim3(kSelThreads), 0, ctx->stream, d_key, n_matches, d_ng,
                       d_par);
    ORB_HIP(hipGetLastError());
    call.fetch(d_ng, ng.data(), 4 * (size_t)nh);
    call.fetch(d_par, par.data(), 4 * (size_t)nh);
    call.fetch(d_good, good.data(), nhn);
    call.fetch(d_p3, P3.data(), 12 * nhn);
    if ((rc = call.finish())) return rc;
    for (int i = 0; i < nh; ++i) {
        out->n_good[i] = ng[i];
        out->parallax[i] = par[i];
    }
    int best = -1;
    if (model == ORBGPU_INIT_MODEL_H) {  // :853-910
        int bestGood = 0, secondBestGood = 0;
        float bestParallax = -1;
        for (int i = 0; i < nh; ++i) {
            if (ng[i] > bestGood) {
                secondBestGood = bestGood;
                bestGood = ng[i];
                best = i;
                bestParallax = par[i];
            } else if (ng[i] > secondBestGood) {
                secondBestGood = ng[i];
            }
        }
        out->ok = secondBestGood < 0.75 * bestGood && bestParallax >= min_parallax && bestGood > min_triangulated &&
                  bestGood > 0.9 * N;
    } else {  // :620-690
        const int maxGood = std::max(ng[0], std::max(ng[1], std::max(ng[2], ng[3])));
        const int nMinGood = std::max(static_cast<int>(0.9 * N), min_triangulated);
        int nsimilar = 0;
        for (int i = 0; i < 4; ++i) nsimilar += ng[i] > 0.7 * maxGood ? 1 : 0;
        if (!(maxGood < nMinGood || nsimilar > 1)) {
            for (int i = 0; i < 4; ++i)
                if (maxGood == ng[i]) {  // the first hypothesis reaching maxGood decides
                    best = i;
                    out->ok = par[i] > min_parallax;
                    break;
                }
        }
    }
    out->best = best;
    if (best >= 0) {
        std::memcpy(out->R21, hy[best].R, sizeof(out->R21));
        std::memcpy(out->t21, hy[best].t, sizeof(out->t21));
    }
    if (out->ok) {
        for (int i = 0; i < n_matches; ++i) {
            const unsigned char g = good[(size_t)best * n + i];
            if (!(g & 2)) continue;  // counted by CheckRT: vP3D[first] written
            const int a = pairs[2 * i];
            if (p3d)
                for (int k = 0; k < 3; ++k) p3d[3 * a + k] = P3[3 * ((size_t)best * n + i) + k];
            if (triangulated) triangulated[a] = g & 1;
        }
    }
    return ORBGPU_OK;
}

extern "C" int orbgpu_init_initialize(const float* kp1, int n1, const float* kp2, int n2, const int* matches12,
                                      const float* K, float sigma, int iterations, orbgpu_init_reconstruction* out,
                                      float* rh, int* model, float* p3d, unsigned char* triangulated) {
    if (!kp1 || !kp2 || !matches12 || !K || !out || !rh || !model || n1 < 0 || n2 < 0 || iterations <= 0)
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    std::vector<int> pairs;  // mvMatches12 (:59-72)
    for (int i = 0; i < n1; ++i)
        if (matches12[i] >= 0) {
            if (matches12[i] >= n2) return fail(ORBGPU_ERR_ARG, "match index out of range");
            pairs.push_back(i);
            pairs.push_back(matches12[i]);
        }
    const int N = (int)pairs.size() / 2;
    if (N < 8) return fail(ORBGPU_ERR_ARG, "fewer than 8 matches (the reference's draws need 8)");
    orbgpu_seed_rand_once(0);  // :102
    std::vector<int> sets(8 * (size_t)iterations);
    int rc = orbgpu_init_draw_sets(N, iterations, sets.data());
    if (rc) return rc;
    rc = check_device();
    if (rc) return rc;
    const size_t work_b = orbgpu_init_workspace_bytes(n1, n2);
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const float *d_kp1, *d_kp2;
    const int *d_pairs, *d_sets;
    void* d_work;
    orbgpu_match_pts* d_pts;
    float *d_h21, *d_h12, *d_f21, *d_sh, *d_sf;
    uint8_t *d_ih, *d_if, *d_pick;
    const size_t it = (size_t)iterations;
    const size_t pick_b = 16 + 72 + 2 * (size_t)N;  // init_pick_kernel's packed read-back
    rc = call.run([&](HostCall& A) {
        d_kp1 = A.inout(kp1, 2 * (size_t)n1, 2 * (size_t)std::max(n1, 1));
        d_kp2 = A.inout(kp2, 2 * (size_t)n2, 2 * (size_t)std::max(n2, 1));
        d_pairs = A.in(pairs.data(), 2 * (size_t)N);
        d_sets = A.in(sets.data(), sets.size());
        d_work = A.out<uint8_t>(std::max<size_t>(work_b, 16));
        d_pts = A.out<orbgpu_match_pts>((size_t)N);
        d_h21 = A.out<float>(9 * it);
        d_h12 = A.out<float>(9 * it);
        d_f21 = A.out<float>(9 * it);
        d_sh = A.out<float>(it);
        d_sf = A.out<float>(it);
        d_ih = A.out<uint8_t>(it * N);
        d_if = A.out<uint8_t>(it * N);
        d_pick = A.out<uint8_t>(pick_b);
    });
    if (rc) return rc;
    // FindHomography / FindFundamental (:160-269): every iteration's hypotheses and scores
    rc = orbgpu_init_hypotheses_batch_device(d_kp1, n1, d_kp2, n2, d_pairs, N, d_sets, iterations, d_work, d_pts,
                                             d_h21, d_h12, d_f21, ctx->stream);
    if (!rc)
        rc = orbgpu_init_check_both_batch_device(d_pts, N, d_h21, d_h12, iterations, d_f21, iterations, sigma, d_sh,
                                                 d_ih, d_sf, d_if, ctx->stream);
    if (rc) return rc;
    // the kept iteration of both models, their matrices and inlier flags in
    // one read-back (init_pick_kernel; the host chose between them after a
    // first read-back of all scores before)
    hipLaunchKernelGGL(init_pick_kernel, dim3(1), dim3(256), 0, ctx->stream, d_sh, d_sf, iterations, d_h21, d_f21,
                       d_ih, d_if, N, d_pick);
    ORB_HIP(hipGetLastError());
    std::vector<uint8_t> pick(pick_b);
    call.fetch(d_pick, pick.data(), pick_b);
    if ((rc = call.finish())) return rc;
    int hdr[4];
    std::memcpy(hdr, pick.data(), 16);
    const int bh = hdr[0], bf = hdr[1];
    float SH, SF;
    std::memcpy(&SH, &hdr[2], 4);
    std::memcpy(&SF, &hdr[3], 4);
    const float RH = SH / (SH + SF);  // :140 (NaN when both are 0: ReconstructF, as the reference)
    const bool useH = RH > 0.40;
    float M[9];
    std::memcpy(M, pick.data() + 16 + (useH ? 0 : 36), 36);
    std::vector<unsigned char> inl(pick.begin() + 16 + 72 + (useH ? 0 : N), pick.begin() + 16 + 72 + (useH ? N : 2 * N));
    const int best = useH ? bh : bf;
    (void)best;
    *rh = RH;
    *model = useH ? ORBGPU_INIT_MODEL_H : ORBGPU_INIT_MODEL_F;
    // (no kept iteration: the reference reconstructs from an empty H/F with no inliers -> false)
    return orbgpu_init_reconstruct(*model, kp1, n1, kp2, n2, pairs.data(), N, inl.data(), M, K, sigma, 1.0f, 50, out,
                                   p3d, triangulated);
}
