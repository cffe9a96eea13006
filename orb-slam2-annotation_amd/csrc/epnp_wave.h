// epnp_wave.h -- EPnP (PnPsolver::compute_pose and helpers,
// src/PnPsolver.cpp:423-1080) for a GROUP of G lanes working together
// (G = 16: four minimal-set hypotheses per wave; G = 64: Refine over all
// inliers on one wave).  Same spec as the one-thread epnp.h (control points,
// sign normalisation, canonical null space, three beta approximations each
// refined by 5 Gauss-Newton steps with the reference's qr_solve, the
// minimum-error choice); what changes is who computes what:
//   * every per-correspondence loop (centroid, covariance, M^T M, the camera
//     centroid and ABt of compute_R_and_t, the reprojection error) is split
//     over the group's lanes and reduced on DPP (group_sum.h);
//   * M^T M is assembled from 40 group sums (its 3x3 blocks are fu^2,
//     fv^2, fu, fv multiples of sums of alpha_k alpha_l weighted by 1,
//     (uc - u), (vc - v) and their squares) and its eigenvectors come from a
//     one-sided Jacobi with the 12 rows on 12 lanes (lane r also carries
//     row r of V; jacobi_group.h: round-robin order, six disjoint column
//     pairs per round, null columns skipped); a column pair's three dot
//     products are group reductions;
//   * the dense 3x3 / 6xk pieces run redundantly on every lane (identical
//     inputs, identical results, no broadcast needed); L (6x10) and the four
//     null-space vectors live in the group's LDS scratch.
// Reduction order differs from the sequential sums of epnp.h, so results
// agree with the oracle to the pose tolerance of tests/test_pnp.py, like
// epnp.h does.  (Round 2: one thread per hypothesis, 512 VGPRs and 2.9 KB of
// scratch per thread, 2.2 ms per 16-solver batch.)
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "epnp.h"
#include "group_sum.h"
#include "jacobi_group.h"
#include "jacobi_lds.h"

namespace orbgpu {
namespace epnp {

// EPNP_STAMPS (diagnostic build only, tools/epnp_stamps.py): lane 0 of a
// chosen group records s_memtime at each phase boundary
#ifdef EPNP_STAMPS
#define EPNP_T(k)                                                        \
    do {                                                                 \
        if (stamps && r == 0) stamps[k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define EPNP_T(k) ((void)stamps)
#endif

// per-group LDS scratch (doubles)
constexpr int kWaveScratch = 144 + 48 + 60;

template <int G>
__device__ __forceinline__ double gsum(double x) {
    return group_sum_dpp<G>(x);
}

// maximum over the lane's 16-lane row
__device__ __forceinline__ double gmax16(double x) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) x = fmax(x, __shfl_xor(x, o, 16));
    return x;
}

// LDS writes of the group visible to its other lanes (one wave: in-order LDS,
// so a counter wait and a wave barrier suffice; no block barrier, so a single
// wave of a larger block can run this)
#define EPNP_GROUP_SYNC()                          \
    do {                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);        \
        __builtin_amdgcn_wave_barrier();           \
    } while (0)

// canonicalize_null_space (epnp.h) for k null vectors held as ut4[c] = ut row
// 11 - c, on one lane, with its small matrices in LDS (scr: >= 80 doubles) so
// they cost no registers
__device__ inline void canonicalize_null_space4(double* ut4, int k, double* scr) {
    double* A = scr;       // k x 2k  (row stride 8)
    double* B = scr + 32;  // 12 x k  (row stride 4)
    for (int i = 0; i < k; ++i)  // [W^T V | I]
        for (int j = 0; j < k; ++j) {
            double acc = 0.0;
            for (int r = 0; r < 12; ++r) acc += null_w(r, i) * ut4[12 * j + r];
            A[8 * i + j] = acc;
            A[8 * i + k + j] = i == j ? 1.0 : 0.0;
        }
    for (int c = 0; c < k; ++c) {  // Gauss-Jordan with partial pivoting
        int p = c;
        for (int r = c + 1; r < k; ++r)
            if (fabs(A[8 * r + c]) > fabs(A[8 * p + c])) p = r;
        if (A[8 * p + c] == 0.0) return;  // degenerate: keep the eigenvectors
        if (p != c)
            for (int j = 0; j < 2 * k; ++j) {
                const double tmp = A[8 * c + j];
                A[8 * c + j] = A[8 * p + j];
                A[8 * p + j] = tmp;
            }
        const double inv = 1.0 / A[8 * c + c];
        for (int j = 0; j < 2 * k; ++j) A[8 * c + j] *= inv;
        for (int r = 0; r < k; ++r)
            if (r != c) {
                const double f = A[8 * r + c];
                for (int j = 0; j < 2 * k; ++j) A[8 * r + j] -= f * A[8 * c + j];
            }
    }
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < k; ++c) {
            double acc = 0.0;
            for (int j = 0; j < k; ++j) acc += ut4[12 * j + r] * A[8 * j + k + c];
            B[4 * r + c] = acc;
        }
    for (int c = 0; c < k; ++c) {  // modified Gram-Schmidt, columns in order
        for (int j = 0; j < c; ++j) {
            double d = 0.0;
            for (int r = 0; r < 12; ++r) d += B[4 * r + j] * B[4 * r + c];
            for (int r = 0; r < 12; ++r) B[4 * r + c] -= d * B[4 * r + j];
        }
        double nrm = 0.0;
        for (int r = 0; r < 12; ++r) nrm += B[4 * r + c] * B[4 * r + c];
        nrm = sqrt(nrm);
        for (int r = 0; r < 12; ++r) B[4 * r + c] /= nrm;
    }
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < 12; ++r) ut4[12 * c + r] = B[4 * r + c];
}

// r = the lane's index in its group; lds = the group's kWaveScratch doubles;
// jac (G = 64 only, optional): JacobiLds<12, 12>::kDoubles of LDS for the
// wave-parallel 12 x 12 decomposition.  Every lane of the group returns the
// same pose and error.
template <int G, class Src>
__device__ double compute_pose_group(const Src& src, const Camera& cam, Pose& out, int r, double* lds,
                                     unsigned long long* stamps = nullptr, double* jac = nullptr) {
    const int n = src.count();
    EPNP_T(0);
    double* s_mtm = lds;        // 12 x 12
    double* s_ut4 = lds + 144;  // 4 x 12: null vectors, ut row 11 - c
    double* s_L = lds + 192;    // 6 x 10
    double cws[4][3];
    // choose_control_points (:423-455)
    {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        for (int i = r; i < n; i += G) {
            double pw[3], u, v;
            src.get(i, pw, u, v);
            a0 += pw[0];
            a1 += pw[1];
            a2 += pw[2];
        }
        cws[0][0] = gsum<G>(a0) / n;
        cws[0][1] = gsum<G>(a1) / n;
        cws[0][2] = gsum<G>(a2) / n;
    }
    {
        double c[6] = {0, 0, 0, 0, 0, 0};  // xx xy xz yy yz zz
        for (int i = r; i < n; i += G) {
            double pw[3], u, v;
            src.get(i, pw, u, v);
            const double d0 = pw[0] - cws[0][0], d1 = pw[1] - cws[0][1], d2 = pw[2] - cws[0][2];
            c[0] += d0 * d0;
            c[1] += d0 * d1;
            c[2] += d0 * d2;
            c[3] += d1 * d1;
            c[4] += d1 * d2;
            c[5] += d2 * d2;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) c[k] = gsum<G>(c[k]);
        double c3[9] = {c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]};
        double dc[3], uct[9];
        sym_eig_desc<3>(c3, dc, uct);
        for (int i = 0; i < 3; ++i) {  // spec: largest-magnitude component positive
            int m = 0;
            for (int j = 1; j < 3; ++j)
                if (fabs(uct[3 * i + j]) > fabs(uct[3 * i + m])) m = j;
            if (uct[3 * i + m] < 0)
                for (int j = 0; j < 3; ++j) uct[3 * i + j] = -uct[3 * i + j];
        }
        for (int i = 1; i < 4; ++i) {
            const double k = sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; ++j) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
        }
    }
    EPNP_T(1);
    // compute_barycentric_coordinates (:457-481): CC_inv = pinv(CC)
    double ci[9];
    {
        double cc[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        double s[3], v[9];
        svd_hestenes<3, 3>(cc, s, v);
        const double thr = fmax(fmax(s[0], s[1]), s[2]) * 2.220446049250313e-16 * 3;
        for (int rr = 0; rr < 3; ++rr)
            for (int c = 0; c < 3; ++c) {
                double acc = 0.0;
                for (int j = 0; j < 3; ++j)
                    if (s[j] > thr) acc += v[rr * 3 + j] * cc[c * 3 + j] / (s[j] * s[j]);
                ci[rr * 3 + c] = acc;
            }
    }
    auto alphas = [&](const double* pw, double* a) {
        for (int j = 0; j < 3; ++j)
            a[1 + j] = ci[3 * j] * (pw[0] - cws[0][0]) + ci[3 * j + 1] * (pw[1] - cws[0][1]) +
                       ci[3 * j + 2] * (pw[2] - cws[0][2]);
        a[0] = 1.0f - a[1] - a[2] - a[3];
    };
    EPNP_T(2);
    // Minimal sets (n = 4, G = 16): M is 8 x 12, so null(M) -- the span of
    // the four smallest eigenvectors of M^T M -- is at least 4-dimensional,
    // and the canonical basis of the spec (Gram-Schmidt of V (W^T V)^-1, V any
    // basis, canonicalize_null_space) is the Gram-Schmidt of the unique N
    // with M N = 0 and W^T N = I.  So N comes from one 12 x 12 solve, [M; W^T]
    // N = [0; I], by Gauss-Jordan with the rows on the group's lanes (pivot
    // = the row with the largest |entry| in the column, found by a row
    // reduction; the pivot row broadcast by shuffles), instead of the 12 x 12
    // eigen-decomposition: the same vectors up to rounding, for ~40x fewer
    // instructions.  A group whose system is (near-)singular (M of rank < 8:
    // degenerate points) makes the wave take the eigen path below.
    bool need_eig = true;
    if constexpr (G == 16) {
        if (n == 4) {
            double row[16];  // 12 coefficients | 4 right-hand sides
#pragma unroll
            for (int j = 0; j < 16; ++j) row[j] = 0.0;
            if (r < 8) {  // fill_M (:483-497): rows 2i, 2i+1 of correspondence i
                double pw[3], u, v, a[4];
                src.get(r >> 1, pw, u, v);
                alphas(pw, a);
                const bool second = r & 1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    row[3 * j] = second ? 0.0 : a[j] * cam.fu;
                    row[3 * j + 1] = second ? a[j] * cam.fv : 0.0;
                    row[3 * j + 2] = second ? a[j] * (cam.vc - v) : a[j] * (cam.uc - u);
                }
            } else if (r < 12) {  // W^T row c, right-hand side e_c
#pragma unroll
                for (int j = 0; j < 12; ++j) row[j] = null_w(j, r - 8);
#pragma unroll
                for (int c = 0; c < 4; ++c) row[12 + c] = (r - 8) == c ? 1.0 : 0.0;
            }
            double amax = 0.0;
#pragma unroll
            for (int j = 0; j < 12; ++j) amax = fmax(amax, fabs(row[j]));
            const double scale = gmax16(amax);
            const int g0 = (int)(threadIdx.x & 63) & ~15;
            bool used = r >= 12, degenerate = false;
            int my_col = -1;
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                // pivot: the unused row with the largest |row[k]| (ties: lowest lane)
                const double av = used ? -1.0 : fabs(row[k]);
                double best = av;
                int bl = r;
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const double ob = __shfl_xor(best, o, 16);
                    const int ol = __shfl_xor(bl, o, 16);
                    if (ob > best || (ob == best && ol < bl)) {
                        best = ob;
                        bl = ol;
                    }
                }
                degenerate |= !(best > 1e-12 * scale);
                double prow[16];
#pragma unroll
                for (int j = k; j < 16; ++j) prow[j] = __shfl(row[j], g0 + bl, 64);
                if (r == bl) {
                    used = true;
                    my_col = k;
                } else if (r < 12) {
                    const double f = row[k] / prow[k];
#pragma unroll
                    for (int j = k; j < 16; ++j) row[j] = fma(-f, prow[j], row[j]);
                }
            }
            // the pivot row of column k holds x_k: N[k][c] = rhs[c] / diag
            double nv[4];
            double dk = 1.0;
#pragma unroll
            for (int k = 0; k < 12; ++k)
                if (my_col == k) dk = row[k];
#pragma unroll
            for (int c = 0; c < 4; ++c) nv[c] = my_col >= 0 ? row[12 + c] / dk : 0.0;
            // modified Gram-Schmidt over the columns, in order (row order is a permutation: sums are order-free
            // up to rounding)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int j = 0; j < c; ++j) {
                    const double d = gsum<16>(nv[j] * nv[c]);
                    nv[c] = fma(-d, nv[j], nv[c]);
                }
                const double nrm = sqrt(gsum<16>(nv[c] * nv[c]));
                nv[c] = nv[c] / nrm;
            }
            if (my_col >= 0)
#pragma unroll
                for (int c = 0; c < 4; ++c) s_ut4[12 * c + my_col] = nv[c];
            need_eig = __any(degenerate);
            EPNP_GROUP_SYNC();
        }
    }
    if (need_eig) {
    // M^T M (fill_M :483-497, cvMulTransposed): per (k <= l) sums of a_k a_l times
    // 1, (uc - u), (vc - v), (uc - u)^2 + (vc - v)^2
    {
        double S1[10], S2[10], S3[10], S4[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) S1[q] = S2[q] = S3[q] = S4[q] = 0.0;
        for (int i = r; i < n; i += G) {
            double pw[3], u, v, a[4];
            src.get(i, pw, u, v);
            alphas(pw, a);
            const double du = cam.uc - u, dv = cam.vc - v, dd = du * du + dv * dv;
            int q = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = k; l < 4; ++l, ++q) {
                    const double aa = a[k] * a[l];
                    S1[q] += aa;
                    S2[q] += aa * du;
                    S3[q] += aa * dv;
                    S4[q] += aa * dd;
                }
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            S1[q] = gsum<G>(S1[q]);
            S2[q] = gsum<G>(S2[q]);
            S3[q] = gsum<G>(S3[q]);
            S4[q] = gsum<G>(S4[q]);
        }
        if (r == 0) {
            const double fu = cam.fu, fv = cam.fv;
            int q = 0;
            for (int k = 0; k < 4; ++k)
                for (int l = k; l < 4; ++l, ++q) {
                    const double blk[9] = {fu * fu * S1[q], 0.0, fu * S2[q], 0.0, fv * fv * S1[q], fv * S3[q],
                                           fu * S2[q], fv * S3[q], S4[q]};
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j) {
                            s_mtm[(3 * k + i) * 12 + 3 * l + j] = blk[3 * i + j];
                            s_mtm[(3 * l + j) * 12 + 3 * k + i] = blk[3 * i + j];
                        }
                }
        }
    }
    EPNP_GROUP_SYNC();
    EPNP_T(3);
    // eigenvectors of M^T M: one-sided Jacobi on the symmetric PSD matrix
    if (G == 64 && jac != nullptr) {
        // a whole wave on one matrix (Refine): the six disjoint pairs of a
        // round on six 8-lane groups, A and V in LDS (jacobi_lds.h)
        using J = JacobiLds<12, 12>;
        double* A = jac;
        double* V = jac + J::M * J::NRP;
        double* nrm = V + J::M * J::NVP;
        J::init(A, V, r, [&](int rr, int c) { return s_mtm[rr * 12 + c]; });
        const int sweeps = J::run(A, V, nrm, r);
#ifdef EPNP_STAMPS
        if (stamps && r == 0) stamps[16] = (unsigned long long)sweeps;
#else
        (void)sweeps;
#endif
        double lam[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) lam[j] = sqrt(nrm[j]);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            int rank = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) rank += (lam[i] > lam[j]) || (i < j && lam[i] == lam[j]);
            if (rank >= 8 && r < 12) s_ut4[12 * (11 - rank) + r] = V[j * J::NVP + r];
        }
    } else {  // rows on lanes (jacobi_group.h)
        double a[12], v[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            a[c] = r < 12 ? s_mtm[r * 12 + c] : 0.0;
            v[c] = (r == c) ? 1.0 : 0.0;
        }
        // the rows sit on lanes 0..11 and every other lane holds zeros, so
        // the 16-lane row sum IS the group sum (the cross-row terms add +0):
        // a wave-wide group (Refine, G = 64) runs its sweeps on DPP row sums
        // alone instead of two ds_bpermute round trips per reduction
        const int sweeps = hestenes_group<12, (G > 16 ? 16 : G)>(a, v);
#ifdef EPNP_STAMPS
        if (stamps && r == 0) stamps[16] = (unsigned long long)sweeps;
#else
        (void)sweeps;
#endif
        double lam[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) lam[j] = sqrt(gsum<G>(a[j] * a[j]));
        // descending order, stable (sym_eig_desc's insertion sort); the four last ranks
        // are the null-space vectors: rank 11 - c -> ut4[c]
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            int rank = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) rank += (lam[i] > lam[j]) || (i < j && lam[i] == lam[j]);
            if (rank >= 8 && r < 12) s_ut4[12 * (11 - rank) + r] = v[j];
        }
    }
    EPNP_GROUP_SYNC();
    EPNP_T(4);
    {
        const int k = 12 - 2 * n;
        if (k > 0 && r == 0) canonicalize_null_space4(s_ut4, k < 4 ? k : 4, s_mtm);  // M^T M is consumed
    }
    EPNP_GROUP_SYNC();
    }  // need_eig
    EPNP_T(5);
    // compute_L_6x10 (:863-898), compute_rho (:900-908)
    double rho[6];
    if (r == 0) {
        double dv[4][6][3];
        for (int i = 0; i < 4; ++i) {
            const double* vv = s_ut4 + 12 * i;
            int a = 0, b = 1;
            for (int j = 0; j < 6; ++j) {
                for (int k = 0; k < 3; ++k) dv[i][j][k] = vv[3 * a + k] - vv[3 * b + k];
                if (++b > 3) {
                    ++a;
                    b = a + 1;
                }
            }
        }
        for (int i = 0; i < 6; ++i) {
            double* row = s_L + 10 * i;
            row[0] = dot3(dv[0][i], dv[0][i]);
            row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
            row[2] = dot3(dv[1][i], dv[1][i]);
            row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
            row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
            row[5] = dot3(dv[2][i], dv[2][i]);
            row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
            row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
            row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
            row[9] = dot3(dv[3][i], dv[3][i]);
        }
    }
    rho[0] = dist2(cws[0], cws[1]);
    rho[1] = dist2(cws[0], cws[2]);
    rho[2] = dist2(cws[0], cws[3]);
    rho[3] = dist2(cws[1], cws[2]);
    rho[4] = dist2(cws[1], cws[3]);
    rho[5] = dist2(cws[2], cws[3]);
    EPNP_GROUP_SYNC();
    EPNP_T(6);
    const double* L = s_L;
    auto gauss_newton = [&](double* betas) {  // :942-963 + compute_A_and_b_gauss_newton :910-940
        double x[4] = {0.0, 0.0, 0.0, 0.0};  // gauss_newton's x: kept by a singular qr_solve
        for (int it = 0; it < 5; ++it) {
            double A[24], b[6];
            for (int i = 0; i < 6; ++i) {
                const double* rr = L + 10 * i;
                double* a = A + 4 * i;
                a[0] = 2 * rr[0] * betas[0] + rr[1] * betas[1] + rr[3] * betas[2] + rr[6] * betas[3];
                a[1] = rr[1] * betas[0] + 2 * rr[2] * betas[1] + rr[4] * betas[2] + rr[7] * betas[3];
                a[2] = rr[3] * betas[0] + rr[4] * betas[1] + 2 * rr[5] * betas[2] + rr[8] * betas[3];
                a[3] = rr[6] * betas[0] + rr[7] * betas[1] + rr[8] * betas[2] + 2 * rr[9] * betas[3];
                b[i] = rho[i] - (rr[0] * betas[0] * betas[0] + rr[1] * betas[0] * betas[1] +
                                 rr[2] * betas[1] * betas[1] + rr[3] * betas[0] * betas[2] +
                                 rr[4] * betas[1] * betas[2] + rr[5] * betas[2] * betas[2] +
                                 rr[6] * betas[0] * betas[3] + rr[7] * betas[1] * betas[3] +
                                 rr[8] * betas[2] * betas[3] + rr[9] * betas[3] * betas[3]);
            }
            qr_solve_6x4(A, b, x);
            for (int i = 0; i < 4; ++i) betas[i] += x[i];
        }
    };
    // compute_R_and_t (:735-745): per-correspondence sums over the group
    // (Serial = false) or over all correspondences on the calling lane
    // (Serial = true: the minimal sets, one beta approximation per lane)
    // Mode 0: the group's lanes (stride G, group reductions); 1: the calling
    // lane alone; 2: the lane's 16-lane row (stride 16, row reductions)
    auto r_and_t_impl = [&](const double* betas, Pose& P, auto mode_tag) -> double {
        constexpr int Mode = decltype(mode_tag)::value;
        const int i0 = Mode == 0 ? r : Mode == 1 ? 0 : (r & 15), di = Mode == 0 ? G : Mode == 1 ? 1 : 16;
        auto red = [&](double x) { return Mode == 0 ? gsum<G>(x) : Mode == 1 ? x : gsum<16>(x); };
        double ccs[4][3];
        for (int i = 0; i < 4; ++i) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; ++i) {
            const double* vv = s_ut4 + 12 * i;
            for (int j = 0; j < 4; ++j)
                for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * vv[3 * j + k];
        }
        auto pc_of = [&](const double* pw, double* pc) {
            double a[4];
            alphas(pw, a);
            for (int j = 0; j < 3; ++j)
                pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        };
        {  // solve_for_sign (:715-733): the sign of point 0's depth
            double pw[3], u, v, pc[3];
            src.get(0, pw, u, v);
            pc_of(pw, pc);
            if (pc[2] < 0.0)
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 3; ++j) ccs[i][j] = -ccs[i][j];
        }
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = i0; i < n; i += di) {
            double pw[3], u, v, pc[3];
            src.get(i, pw, u, v);
            pc_of(pw, pc);
            for (int j = 0; j < 3; ++j) {
                pc0[j] += pc[j];
                pw0[j] += pw[j];
            }
        }
        for (int j = 0; j < 3; ++j) {
            pc0[j] = red(pc0[j]) / n;
            pw0[j] = red(pw0[j]) / n;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = i0; i < n; i += di) {
            double pw[3], u, v, pc[3];
            src.get(i, pw, u, v);
            pc_of(pw, pc);
            for (int j = 0; j < 3; ++j) {
                abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) abt[k] = red(abt[k]);
        double s[3], vv[9];
        svd_hestenes<3, 3>(abt, s, vv);  // abt columns = U_j s_j
        double U[9];
        for (int rr = 0; rr < 3; ++rr)
            for (int c = 0; c < 3; ++c) U[rr * 3 + c] = s[c] > 0.0 ? abt[rr * 3 + c] / s[c] : 0.0;
        double* R = P.R;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[3 * i + j] = dot3(U + 3 * i, vv + 3 * j);
        const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                           R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
        if (det < 0) {
            R[6] = -R[6];
            R[7] = -R[7];
            R[8] = -R[8];
        }
        P.t[0] = pc0[0] - dot3(R, pw0);
        P.t[1] = pc0[1] - dot3(R + 3, pw0);
        P.t[2] = pc0[2] - dot3(R + 6, pw0);
        double sum2 = 0.0;
        for (int i = i0; i < n; i += di) {
            double pw[3], u, v;
            src.get(i, pw, u, v);
            const double Xc = dot3(R, pw) + P.t[0], Yc = dot3(R + 3, pw) + P.t[1];
            const double inv_Zc = 1.0 / (dot3(R + 6, pw) + P.t[2]);
            const double ue = cam.uc + cam.fu * Xc * inv_Zc, ve = cam.vc + cam.fv * Yc * inv_Zc;
            sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
        return red(sum2) / n;
    };
    auto r_and_t = [&](const double* betas, Pose& P) { return r_and_t_impl(betas, P, std::integral_constant<int, 0>{}); };
    double best_err;
    auto keep = [&](double e, const Pose& P, bool first) {  // N = 1; err[2] < err[N] -> 2; err[3] < err[N] -> 3
        if (first || e < best_err) {
            best_err = e;
            out = P;
        }
    };
    if constexpr (G == 16 || G == 64) {
        // The three beta approximations side by side: on lanes 0, 1, 2 of a
        // 16-lane group (minimal sets: compute_R_and_t over the n
        // correspondences on the lane), or on rows 0, 1, 2 of the wave
        // (Refine: compute_R_and_t with the row's 16 lanes over all
        // correspondences); the other lanes / row repeat the third.  Then the
        // reference's choice (1, then 2 or 3 if strictly better, in order).
        // The 6 x 4 / 6 x 3 systems of approximations 1 and 2 are solved as
        // 6 x 5 with zero columns: the Jacobi skips every pair with a zero
        // column and the pseudo-inverse gives them zero, so the solution is
        // bit for bit the smaller system's.
        const int ap = min(G == 16 ? r : (r >> 4), 2);
        double l[30], b5[5], B[4];
        for (int i = 0; i < 6; ++i) {
            const double* Lr = L + 10 * i;
            l[5 * i] = Lr[0];
            l[5 * i + 1] = Lr[1];
            l[5 * i + 2] = ap == 0 ? Lr[3] : Lr[2];
            l[5 * i + 3] = ap == 0 ? Lr[6] : ap == 1 ? 0.0 : Lr[3];
            l[5 * i + 4] = ap == 2 ? Lr[4] : 0.0;
        }
        if (G == 64 && jac != nullptr) {
            // Refine: each row's 6 x 5 solve on its own 12 lanes (three 4-lane
            // column pairs per round-robin round, jacobi_lds.h), A and V in
            // LDS -- rows 0..2 in the 12 x 12 decomposition's area, row 3 (a
            // duplicate of approximation 3) in the consumed M^T M area; on one
            // lane each the sequential Jacobi took ~55 k cycles
            using JB = JacobiLds<5, 6, 4, 16>;
            static_assert(3 * JB::kDoubles <= JacobiLds<12, 12>::kDoubles && JB::kDoubles <= 144, "LDS areas");
            const int grp = r >> 4;
            double* JA = grp < 3 ? jac + grp * JB::kDoubles : lds;
            double* JV = JA + JB::M * JB::NRP;
            double* jn = JV + JB::M * JB::NVP;
            JB::init(JA, JV, r, [](int, int) { return 0.0; });
            // l[] into A with constant indices only (a dynamically indexed l went to scratch)
#pragma unroll
            for (int e = 0; e < 30; ++e)
                if ((e & 15) == (r & 15)) JA[(e % 5) * JB::NRP + e / 5] = l[e];
            JB::sync();
            JB::run(JA, JV, jn, r);
            double sv[5], smax = 0.0, y[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                sv[j] = sqrt(jn[j]);
                smax = fmax(smax, sv[j]);
            }
            const double thr = smax * 2.220446049250313e-16 * 6;
#pragma unroll
            for (int j = 0; j < 5; ++j) {  // y = Sigma^+ U^T rho, U_j = a_j / s_j (svd_solve's pinv)
                double d = 0.0;
                if (sv[j] > thr) {
#pragma unroll
                    for (int rr = 0; rr < 6; ++rr) d += JA[j * JB::NRP + rr] * rho[rr];
                    d /= sv[j] * sv[j];
                }
                y[j] = d;
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                double acc = 0.0;
#pragma unroll
                for (int j = 0; j < 5; ++j) acc += JV[j * JB::NVP + i] * y[j];
                b5[i] = acc;
            }
        } else {
            svd_solve<6, 5>(l, rho, b5);
        }
        if (ap == 0) {  // find_betas_approx_1 (:747-781)
            if (b5[0] < 0) {
                B[0] = sqrt(-b5[0]);
                B[1] = -b5[1] / B[0];
                B[2] = -b5[2] / B[0];
                B[3] = -b5[3] / B[0];
            } else {
                B[0] = sqrt(b5[0]);
                B[1] = b5[1] / B[0];
                B[2] = b5[2] / B[0];
                B[3] = b5[3] / B[0];
            }
        } else {  // find_betas_approx_2 (:783-815) / _3 (:817-851)
            if (b5[0] < 0) {
                B[0] = sqrt(-b5[0]);
                B[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
            } else {
                B[0] = sqrt(b5[0]);
                B[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
            }
            if (b5[1] < 0) B[0] = -B[0];
            B[2] = ap == 2 ? b5[3] / B[0] : 0.0;
            B[3] = 0.0;
        }
        EPNP_T(7);
        gauss_newton(B);
        EPNP_T(8);
        Pose P;
        double e;
        if constexpr (G == 16)
            e = r_and_t_impl(B, P, std::integral_constant<int, 1>{});
        else
            e = r_and_t_impl(B, P, std::integral_constant<int, 2>{});
        EPNP_T(15);
        const int base = G == 16 ? ((int)(threadIdx.x & 63) & ~15) : 0, step = G == 16 ? 1 : 16;
        const double e0 = __shfl(e, base, 64), e1 = __shfl(e, base + step, 64), e2 = __shfl(e, base + 2 * step, 64);
        int pick = 0;
        double best = e0;
        if (e1 < best) {
            best = e1;
            pick = 1;
        }
        if (e2 < best) {
            best = e2;
            pick = 2;
        }
        const int src_lane = base + pick * step;
        for (int k = 0; k < 9; ++k) out.R[k] = __shfl(P.R[k], src_lane, 64);
        for (int k = 0; k < 3; ++k) out.t[k] = __shfl(P.t[k], src_lane, 64);
        return best;
    } else {
    {  // find_betas_approx_1 (:747-781)
        double l[24], b4[4], B[4];
        for (int i = 0; i < 6; ++i) {
            l[4 * i] = L[10 * i];
            l[4 * i + 1] = L[10 * i + 1];
            l[4 * i + 2] = L[10 * i + 3];
            l[4 * i + 3] = L[10 * i + 6];
        }
        svd_solve<6, 4>(l, rho, b4);
        EPNP_T(7);
        if (b4[0] < 0) {
            B[0] = sqrt(-b4[0]);
            B[1] = -b4[1] / B[0];
            B[2] = -b4[2] / B[0];
            B[3] = -b4[3] / B[0];
        } else {
            B[0] = sqrt(b4[0]);
            B[1] = b4[1] / B[0];
            B[2] = b4[2] / B[0];
            B[3] = b4[3] / B[0];
        }
        gauss_newton(B);
        EPNP_T(8);
        Pose P;
        const double e = r_and_t(B, P);
        keep(e, P, true);
    }
    EPNP_T(9);
    {  // find_betas_approx_2 (:783-815)
        double l[18], b3[3], B[4];
        for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 3; ++k) l[3 * i + k] = L[10 * i + k];
        svd_solve<6, 3>(l, rho, b3);
        EPNP_T(10);
        if (b3[0] < 0) {
            B[0] = sqrt(-b3[0]);
            B[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
        } else {
            B[0] = sqrt(b3[0]);
            B[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) B[0] = -B[0];
        B[2] = 0.0;
        B[3] = 0.0;
        gauss_newton(B);
        EPNP_T(11);
        Pose P;
        const double e = r_and_t(B, P);
        keep(e, P, false);
    }
    EPNP_T(12);
    {  // find_betas_approx_3 (:817-851)
        double l[30], b5[5], B[4];
        for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 5; ++k) l[5 * i + k] = L[10 * i + k];
        svd_solve<6, 5>(l, rho, b5);
        EPNP_T(13);
        if (b5[0] < 0) {
            B[0] = sqrt(-b5[0]);
            B[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
        } else {
            B[0] = sqrt(b5[0]);
            B[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) B[0] = -B[0];
        B[2] = b5[3] / B[0];
        B[3] = 0.0;
        gauss_newton(B);
        EPNP_T(14);
        Pose P;
        const double e = r_and_t(B, P);
        keep(e, P, false);
    }
    EPNP_T(15);
    return best_err;
    }
}

}  // namespace epnp
}  // namespace orbgpu
