// epnp.h -- device EPnP (PnPsolver::compute_pose and its helpers,
// src/PnPsolver.cpp:423-1080) in double precision, written for ONE thread.
//
// Correspondences are streamed through a source object (no per-point
// scratch): src.count(), src.get(i, pw[3], u, v).  The pass structure
// follows the reference: control points from the centroid + principal
// directions of the world points (choose_control_points), barycentric
// coordinates (compute_barycentric_coordinates), M^T M accumulated over the
// 2n rows of M (fill_M, cvMulTransposed), its 4 least-eigenvalue vectors
// (cvSVD of M^T M), L_6x10 / rho, three beta approximations each refined
// by 5 Gauss-Newton steps with the reference's Householder qr_solve,
// compute_R_and_t (ccs -> pcs -> solve_for_sign -> Procrustes via SVD of
// ABt) and the minimum mean reprojection error among the three.
//
// The OpenCV SVD calls are restated with Jacobi methods: symmetric
// eigen-decomposition (cyclic Jacobi, eigenvalues sorted descending) for
// the symmetric PSD matrices, one-sided (Hestenes) Jacobi for the general
// ones (cvInvert / cvSolve with CV_SVD, the 3x3 ABt).
#pragma once

#include <hip/hip_runtime.h>

#include "jacobi_group.h"

namespace orbgpu {
namespace epnp {

// cyclic Jacobi on symmetric n x n `a` (row-major, destroyed); eigenvalues
// to w[0..n) and eigenvectors to the ROWS of ut, sorted by descending
// eigenvalue (cvSVD(..., CV_SVD_U_T) of a symmetric PSD matrix).
template <int N>
__host__ __device__ void sym_eig_desc(double* a, double* w, double* ut) {
    double v[N * N];
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) v[i * N + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int i = 0; i < N; ++i) {
            diag += a[i * N + i] * a[i * N + i];
            for (int j = i + 1; j < N; ++j) off += a[i * N + j] * a[i * N + j];
        }
        if (off <= 1e-32 * diag || off == 0.0) break;
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p * N + q];
                if (fabs(apq) < 1e-300) continue;
                const double theta = (a[q * N + q] - a[p * N + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < N; ++k) {
                    const double akp = a[k * N + p], akq = a[k * N + q];
                    a[k * N + p] = c * akp - s * akq;
                    a[k * N + q] = s * akp + c * akq;
                }
                for (int k = 0; k < N; ++k) {
                    const double apk = a[p * N + k], aqk = a[q * N + k];
                    a[p * N + k] = c * apk - s * aqk;
                    a[q * N + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < N; ++k) {
                    const double vkp = v[k * N + p], vkq = v[k * N + q];
                    v[k * N + p] = c * vkp - s * vkq;
                    v[k * N + q] = s * vkp + c * vkq;
                }
            }
    }
    // descending by eigenvalue, stable (the order of an insertion sort that
    // moves an entry before strictly smaller ones): column c goes to rank
    // #{j : w_j > w_c} + #{j < c : w_j == w_c}; selected with constant
    // indices only (a dynamic order[] put a, v, w and ut in scratch memory)
#pragma unroll
    for (int c = 0; c < N; ++c) {
        int rank = 0;
#pragma unroll
        for (int j = 0; j < N; ++j)
            rank += (a[j * N + j] > a[c * N + c]) || (j < c && a[j * N + j] == a[c * N + c]);
#pragma unroll
        for (int r = 0; r < N; ++r)
            if (rank == r) {
                w[r] = a[c * N + c];
#pragma unroll
                for (int k = 0; k < N; ++k) ut[r * N + k] = v[k * N + c];
            }
    }
}

// one-sided Jacobi SVD of m x n `a` (m >= n, row-major): on return the
// columns of a are U_j * sigma_j, sigma in s[], V in v (n x n, row-major)
template <int M, int N>
__host__ __device__ void svd_hestenes(double* a, double* s, double* v) {
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) v[i * N + j] = i == j ? 1.0 : 0.0;
    double fro = 0.0;  // numerically null columns take no rotation (jacobi_group.h)
    for (int k = 0; k < M * N; ++k) fro += a[k] * a[k];
    const double negl = kJacobiNegl * fro;
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool rotated = false;
        // fully unrolled (device): constant indices keep a and v in registers
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    alpha += a[k * N + p] * a[k * N + p];
                    beta += a[k * N + q] * a[k * N + q];
                    gamma += a[k * N + p] * a[k * N + q];
                }
                double c, sn;
                if (!jacobi_rot(alpha, beta, gamma, negl, c, sn)) continue;
                rotated = true;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    const double x = a[k * N + p], y = a[k * N + q];
                    a[k * N + p] = c * x - sn * y;
                    a[k * N + q] = sn * x + c * y;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double x = v[k * N + p], y = v[k * N + q];
                    v[k * N + p] = c * x - sn * y;
                    v[k * N + q] = sn * x + c * y;
                }
            }
        if (!rotated) break;
    }
    for (int j = 0; j < N; ++j) {
        double nrm = 0.0;
        for (int k = 0; k < M; ++k) nrm += a[k * N + j] * a[k * N + j];
        s[j] = sqrt(nrm);
    }
}

// x = pinv(A) b for m x n A (cvSolve(A, b, x, CV_SVD)); A is destroyed
template <int M, int N>
__host__ __device__ void svd_solve(double* A, const double* b, double* x) {
    double s[N], v[N * N];
    svd_hestenes<M, N>(A, s, v);
    double smax = 0.0;
    for (int j = 0; j < N; ++j) smax = fmax(smax, s[j]);
    const double thr = smax * 2.220446049250313e-16 * M;
    double y[N];
    for (int j = 0; j < N; ++j) {  // y = Sigma^+ U^T b, U_j = a_j / s_j
        double d = 0.0;
        if (s[j] > thr) {
            for (int k = 0; k < M; ++k) d += A[k * N + j] * b[k];
            d /= s[j] * s[j];
        }
        y[j] = d;
    }
    for (int i = 0; i < N; ++i) {
        double acc = 0.0;
        for (int j = 0; j < N; ++j) acc += v[i * N + j] * y[j];
        x[i] = acc;
    }
}

__host__ __device__ inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__host__ __device__ inline double dist2(const double* p, const double* q) {
    return (p[0] - q[0]) * (p[0] - q[0]) + (p[1] - q[1]) * (p[1] - q[1]) + (p[2] - q[2]) * (p[2] - q[2]);
}

// PnPsolver::qr_solve (PnPsolver.cpp:955-1047), 6 x 4, A and b destroyed.
// The eta scan is the reference's pointer loop (:975-980): it starts at
// |A[k][k]| and, for i = k+1 .. nr-1, reads the row BEFORE advancing, so it
// covers rows k .. nr-2 and never the last row.  A zero eta is the
// reference's singular return (:982-985): X is left as it is (the caller's
// x persists across the Gauss-Newton iterations, as gauss_newton's does).
__host__ __device__ inline void qr_solve_6x4(double* A, double* b, double* X) {
    constexpr int nr = 6, nc = 4;
    double A1[nc], A2[nc];
    for (int k = 0; k < nc; ++k) {
        double eta = fabs(A[k * nc + k]);
        for (int i = k + 1; i < nr; ++i) {
            const double elt = fabs(A[(i - 1) * nc + k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0.0) return;
        double sum = 0.0;
        const double inv_eta = 1.0 / eta;
        for (int i = k; i < nr; ++i) {
            A[i * nc + k] *= inv_eta;
            sum += A[i * nc + k] * A[i * nc + k];
        }
        double sigma = sqrt(sum);
        if (A[k * nc + k] < 0) sigma = -sigma;
        A[k * nc + k] += sigma;
        A1[k] = sigma * A[k * nc + k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; ++j) {
            double s2 = 0.0;
            for (int i = k; i < nr; ++i) s2 += A[i * nc + k] * A[i * nc + j];
            const double tau = s2 / A1[k];
            for (int i = k; i < nr; ++i) A[i * nc + j] -= tau * A[i * nc + k];
        }
    }
    for (int j = 0; j < nc; ++j) {
        double tau = 0.0;
        for (int i = j; i < nr; ++i) tau += A[i * nc + j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; ++i) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; --i) {
        double sum = 0.0;
        for (int j = i + 1; j < nc; ++j) sum += A[i * nc + j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

struct Camera {
    double fu, fv, uc, vc;
};

// Null-space canonicalisation (spec decision): with n < 6
// correspondences M (2n x 12) has an exact null space of dimension
// k = 12 - 2n (4 for a minimal set) whose eigenvectors cvSVD returns in a
// basis fixed only by rounding noise -- and the beta approximations are not
// invariant to that basis.  Both the oracle and this kernel replace those k
// vectors by the one orthonormal basis Q of the same subspace with W^T Q
// upper triangular (Q = Gram-Schmidt of V (W^T V)^-1) for this fixed,
// exactly representable W.
__host__ __device__ inline double null_w(int i, int j) { return ((i * 7 + j * 13 + i * j * 5 + 3) % 17 - 8) / 8.0; }

__host__ __device__ inline void canonicalize_null_space(double* ut, int k) {
    double V[12][4], A[4][8];
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < 12; ++r) V[r][c] = ut[12 * (11 - c) + r];
    for (int i = 0; i < k; ++i)  // [W^T V | I]
        for (int j = 0; j < k; ++j) {
            double acc = 0.0;
            for (int r = 0; r < 12; ++r) acc += null_w(r, i) * V[r][j];
            A[i][j] = acc;
            A[i][k + j] = i == j ? 1.0 : 0.0;
        }
    for (int c = 0; c < k; ++c) {  // Gauss-Jordan with partial pivoting
        int p = c;
        for (int r = c + 1; r < k; ++r)
            if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (A[p][c] == 0.0) return;  // degenerate: keep the eigenvectors
        if (p != c)
            for (int j = 0; j < 2 * k; ++j) {
                const double tmp = A[c][j];
                A[c][j] = A[p][j];
                A[p][j] = tmp;
            }
        const double inv = 1.0 / A[c][c];
        for (int j = 0; j < 2 * k; ++j) A[c][j] *= inv;
        for (int r = 0; r < k; ++r)
            if (r != c) {
                const double f = A[r][c];
                for (int j = 0; j < 2 * k; ++j) A[r][j] -= f * A[c][j];
            }
    }
    double B[12][4];
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < k; ++c) {
            double acc = 0.0;
            for (int j = 0; j < k; ++j) acc += V[r][j] * A[j][k + c];
            B[r][c] = acc;
        }
    for (int c = 0; c < k; ++c) {  // modified Gram-Schmidt, columns in order
        for (int j = 0; j < c; ++j) {
            double d = 0.0;
            for (int r = 0; r < 12; ++r) d += B[r][j] * B[r][c];
            for (int r = 0; r < 12; ++r) B[r][c] -= d * B[r][j];
        }
        double nrm = 0.0;
        for (int r = 0; r < 12; ++r) nrm += B[r][c] * B[r][c];
        nrm = sqrt(nrm);
        for (int r = 0; r < 12; ++r) B[r][c] /= nrm;
    }
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < 12; ++r) ut[12 * (11 - c) + r] = B[r][c];
}

struct Pose {
    double R[9], t[3];
};

// EPnP over the correspondences of `src`; returns the mean reprojection
// error of the chosen solution (compute_pose, PnPsolver.cpp:523-580)
template <class Src>
__host__ __device__ double compute_pose(const Src& src, const Camera& cam, Pose& out) {
    const int n = src.count();
    double cws[4][3];
    // choose_control_points (:423-455)
    cws[0][0] = cws[0][1] = cws[0][2] = 0.0;
    for (int i = 0; i < n; ++i) {
        double pw[3], u, v;
        src.get(i, pw, u, v);
        for (int j = 0; j < 3; ++j) cws[0][j] += pw[j];
    }
    for (int j = 0; j < 3; ++j) cws[0][j] /= n;
    {
        double c3[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; ++i) {
            double pw[3], u, v;
            src.get(i, pw, u, v);
            const double d[3] = {pw[0] - cws[0][0], pw[1] - cws[0][1], pw[2] - cws[0][2]};
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) c3[r * 3 + c] += d[r] * d[c];
        }
        double dc[3], uct[9];
        sym_eig_desc<3>(c3, dc, uct);
        // spec decision: the principal directions' signs, left
        // to rounding by cvSVD, are fixed -- largest-magnitude component
        // positive -- since the control points and hence EPnP's estimate
        // depend on them
        for (int i = 0; i < 3; ++i) {
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
    // compute_barycentric_coordinates (:457-481): CC_inv = pinv(CC)
    double ci[9];
    {
        double cc[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        double s[3], v[9];
        svd_hestenes<3, 3>(cc, s, v);
        const double thr = fmax(fmax(s[0], s[1]), s[2]) * 2.220446049250313e-16 * 3;
        for (int r = 0; r < 3; ++r)  // pinv = V diag(1/s^2) (U s)^T
            for (int c = 0; c < 3; ++c) {
                double acc = 0.0;
                for (int j = 0; j < 3; ++j)
                    if (s[j] > thr) acc += v[r * 3 + j] * cc[c * 3 + j] / (s[j] * s[j]);
                ci[r * 3 + c] = acc;
            }
    }
    auto alphas = [&](const double* pw, double* a) {
        for (int j = 0; j < 3; ++j)
            a[1 + j] = ci[3 * j] * (pw[0] - cws[0][0]) + ci[3 * j + 1] * (pw[1] - cws[0][1]) +
                       ci[3 * j + 2] * (pw[2] - cws[0][2]);
        a[0] = 1.0f - a[1] - a[2] - a[3];
    };
    // M^T M over the rows of fill_M (:483-497)
    double ut[144];
    {
        double mtm[144];
        for (int k = 0; k < 144; ++k) mtm[k] = 0.0;
        for (int i = 0; i < n; ++i) {
            double pw[3], u, v, a[4];
            src.get(i, pw, u, v);
            alphas(pw, a);
            double r1[12], r2[12];
            for (int k = 0; k < 4; ++k) {
                r1[3 * k] = a[k] * cam.fu;
                r1[3 * k + 1] = 0.0;
                r1[3 * k + 2] = a[k] * (cam.uc - u);
                r2[3 * k] = 0.0;
                r2[3 * k + 1] = a[k] * cam.fv;
                r2[3 * k + 2] = a[k] * (cam.vc - v);
            }
            for (int r = 0; r < 12; ++r)
                for (int c = r; c < 12; ++c) mtm[r * 12 + c] += r1[r] * r1[c] + r2[r] * r2[c];
        }
        for (int r = 0; r < 12; ++r)
            for (int c = 0; c < r; ++c) mtm[r * 12 + c] = mtm[c * 12 + r];
        double d[12];
        sym_eig_desc<12>(mtm, d, ut);
        const int k = 12 - 2 * n;
        if (k > 0) canonicalize_null_space(ut, k < 4 ? k : 4);
    }
    // compute_L_6x10 (:863-898), compute_rho (:900-908)
    double L[60], rho[6];
    {
        double dv[4][6][3];
        for (int i = 0; i < 4; ++i) {
            const double* vv = ut + 12 * (11 - i);
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
            double* row = L + 10 * i;
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
        rho[0] = dist2(cws[0], cws[1]);
        rho[1] = dist2(cws[0], cws[2]);
        rho[2] = dist2(cws[0], cws[3]);
        rho[3] = dist2(cws[1], cws[2]);
        rho[4] = dist2(cws[1], cws[3]);
        rho[5] = dist2(cws[2], cws[3]);
    }
    auto gauss_newton = [&](double* betas) {  // :942-963 + compute_A_and_b_gauss_newton :910-940
        double x[4] = {0.0, 0.0, 0.0, 0.0};  // gauss_newton's x: kept by a singular qr_solve
        for (int it = 0; it < 5; ++it) {
            double A[24], b[6];
            for (int i = 0; i < 6; ++i) {
                const double* r = L + 10 * i;
                double* a = A + 4 * i;
                a[0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
                a[1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
                a[2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
                a[3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
                b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                                 r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                                 r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                                 r[9] * betas[3] * betas[3]);
            }
            qr_solve_6x4(A, b, x);
            for (int i = 0; i < 4; ++i) betas[i] += x[i];
        }
    };
    // compute_R_and_t (:735-745): ccs, pcs (streamed), solve_for_sign,
    // estimate_R_and_t (:636-700), reprojection_error (:612-634)
    auto r_and_t = [&](const double* betas, Pose& P) -> double {
        double ccs[4][3];
        for (int i = 0; i < 4; ++i) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; ++i) {
            const double* vv = ut + 12 * (11 - i);
            for (int j = 0; j < 4; ++j)
                for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * vv[3 * j + k];
        }
        auto pc_of = [&](const double* pw, double* pc) {
            double a[4];
            alphas(pw, a);
            for (int j = 0; j < 3; ++j) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
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
        for (int i = 0; i < n; ++i) {
            double pw[3], u, v, pc[3];
            src.get(i, pw, u, v);
            pc_of(pw, pc);
            for (int j = 0; j < 3; ++j) {
                pc0[j] += pc[j];
                pw0[j] += pw[j];
            }
        }
        for (int j = 0; j < 3; ++j) {
            pc0[j] /= n;
            pw0[j] /= n;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; ++i) {
            double pw[3], u, v, pc[3];
            src.get(i, pw, u, v);
            pc_of(pw, pc);
            for (int j = 0; j < 3; ++j) {
                abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
        double s[3], vv[9];
        svd_hestenes<3, 3>(abt, s, vv);  // abt columns = U_j s_j
        double U[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) U[r * 3 + c] = s[c] > 0.0 ? abt[r * 3 + c] / s[c] : 0.0;
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
        for (int i = 0; i < n; ++i) {
            double pw[3], u, v;
            src.get(i, pw, u, v);
            const double Xc = dot3(R, pw) + P.t[0], Yc = dot3(R + 3, pw) + P.t[1];
            const double inv_Zc = 1.0 / (dot3(R + 6, pw) + P.t[2]);
            const double ue = cam.uc + cam.fu * Xc * inv_Zc, ve = cam.vc + cam.fv * Yc * inv_Zc;
            sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
        return sum2 / n;
    };
    double betas[4][4], err[4];
    Pose Ps[4];
    {  // find_betas_approx_1 (:747-781)
        double l[24], b4[4];
        for (int i = 0; i < 6; ++i) {
            l[4 * i] = L[10 * i];
            l[4 * i + 1] = L[10 * i + 1];
            l[4 * i + 2] = L[10 * i + 3];
            l[4 * i + 3] = L[10 * i + 6];
        }
        svd_solve<6, 4>(l, rho, b4);
        double* B = betas[1];
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
        err[1] = r_and_t(B, Ps[1]);
    }
    {  // find_betas_approx_2 (:783-815)
        double l[18], b3[3];
        for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 3; ++k) l[3 * i + k] = L[10 * i + k];
        svd_solve<6, 3>(l, rho, b3);
        double* B = betas[2];
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
        err[2] = r_and_t(B, Ps[2]);
    }
    {  // find_betas_approx_3 (:817-851)
        double l[30], b5[5];
        for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 5; ++k) l[5 * i + k] = L[10 * i + k];
        svd_solve<6, 5>(l, rho, b5);
        double* B = betas[3];
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
        err[3] = r_and_t(B, Ps[3]);
    }
    int N = 1;
    if (err[2] < err[1]) N = 2;
    if (err[3] < err[N]) N = 3;
    out = Ps[N];
    return err[N];
}

}  // namespace epnp
}  // namespace orbgpu
