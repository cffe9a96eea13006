// pnp_ref.cpp -- C++ restatement of oracle/pnp_ref.py: PnPsolver's EPnP
// (compute_pose, src/PnPsolver.cpp:392-1047) and the loop body of iterate
// with Refine (:224-349) and CheckInliers (:352-386).
//
// TEST INFRASTRUCTURE ONLY.  It follows pnp_ref.py step for step; the
// LAPACK calls of the numpy oracle (eigh, pinv, lstsq, svd) become a Jacobi
// eigen-decomposition and a one-sided Jacobi SVD in double with the same
// cut-offs, so poses agree with the numpy oracle to rounding and the integer
// outcomes (found, consumed, inlier counts) are equal
// (tests/test_oracle_proj_cpp.py).  It exists so the drop-in latency table
// (bench.py DropIn.cpu_oracle) times PnPsolver::iterate in compiled code.
// Parity vs the reference binary: unpinned (OpenCV absent), as pnp_ref.py.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

// one-sided Jacobi SVD of the m x n row-major a (m >= n): on return the
// columns of a are U_j s_j; s[n], v (n x n row-major, columns = V_j)
void svd_jacobi(std::vector<double>& a, int m, int n, std::vector<double>& s, std::vector<double>& v) {
    v.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) v[(size_t)i * n + i] = 1.0;
    // a column whose squared norm is below 1e-28 ||A||_F^2 is numerically
    // null and takes no rotation (an exactly rank-deficient M^T M, e.g. a
    // minimal set's, never meets the relative test otherwise)
    double fro = 0;
    for (double x : a) fro += x * x;
    const double negl = 1e-28 * fro;
    for (int sweep = 0; sweep < 80; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int k = 0; k < m; ++k) {
                    const double x = a[(size_t)k * n + p], y = a[(size_t)k * n + q];
                    al += x * x;
                    be += y * y;
                    ga += x * y;
                }
                if (ga == 0.0 || std::fabs(ga) <= 1e-15 * std::sqrt(al * be) || al <= negl || be <= negl) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
                for (int k = 0; k < m; ++k) {
                    const double x = a[(size_t)k * n + p], y = a[(size_t)k * n + q];
                    a[(size_t)k * n + p] = c * x - sn * y;
                    a[(size_t)k * n + q] = sn * x + c * y;
                }
                for (int k = 0; k < n; ++k) {
                    const double x = v[(size_t)k * n + p], y = v[(size_t)k * n + q];
                    v[(size_t)k * n + p] = c * x - sn * y;
                    v[(size_t)k * n + q] = sn * x + c * y;
                }
            }
        if (!rotated) break;
    }
    s.assign(n, 0.0);
    for (int j = 0; j < n; ++j) {
        double nn = 0;
        for (int k = 0; k < m; ++k) nn += a[(size_t)k * n + j] * a[(size_t)k * n + j];
        s[j] = std::sqrt(nn);
    }
}

// x = pinv(A) b with numpy's cut-off rcond * s_max (lstsq rcond=None: eps * max(m, n))
std::vector<double> lstsq(const std::vector<double>& A, int m, int n, const double* b, double rcond) {
    std::vector<double> a = A, s, v;
    svd_jacobi(a, m, n, s, v);
    const double smax = *std::max_element(s.begin(), s.end());
    std::vector<double> y(n, 0.0), x(n, 0.0);
    for (int j = 0; j < n; ++j) {
        if (!(s[j] > rcond * smax)) continue;
        double d = 0;
        for (int k = 0; k < m; ++k) d += a[(size_t)k * n + j] * b[k];
        y[j] = d / (s[j] * s[j]);
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) x[i] += v[(size_t)i * n + j] * y[j];
    return x;
}

// eigen-decomposition of the symmetric PSD n x n a: eigenvalues descending
// (stable), eigenvectors as the ROWS of ut (np.linalg.eigh + argsort)
void sym_eig_desc(const std::vector<double>& A, int n, std::vector<double>& w, std::vector<double>& ut) {
    std::vector<double> a = A, s, v;
    svd_jacobi(a, n, n, s, v);  // PSD: singular values = eigenvalues, V = eigenvectors
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return s[x] > s[y]; });
    w.resize(n);
    ut.assign((size_t)n * n, 0.0);
    for (int r = 0; r < n; ++r) {
        w[r] = s[order[r]];
        for (int k = 0; k < n; ++k) ut[(size_t)r * n + k] = v[(size_t)k * n + order[r]];
    }
}

// PnPsolver::qr_solve (PnPsolver.cpp:955-1047), 6 x 4.  The eta scan is the
// reference's pointer loop (:975-980): it starts at |A[k][k]| and for
// i = k+1 .. nr-1 reads row i-1 (the pointer advances after the read), so the
// last row never takes part; the column is scaled by *= inv_eta with
// inv_eta = 1./eta (:987-990).  Singular (eta == 0, :982-985): return with X
// untouched.
void qr_solve(double A[6][4], double b[6], double X[4]) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; ++k) {
        double eta = std::fabs(A[k][k]);
        for (int i = k + 1; i < nr; ++i) {
            const double elt = std::fabs(A[i - 1][k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;
        const double inv_eta = 1. / eta;
        double sum = 0;
        for (int i = k; i < nr; ++i) {
            A[i][k] *= inv_eta;
            sum += A[i][k] * A[i][k];
        }
        double sigma = std::sqrt(sum);
        if (A[k][k] < 0) sigma = -sigma;
        A[k][k] += sigma;
        A1[k] = sigma * A[k][k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; ++j) {
            double tau = 0;
            for (int i = k; i < nr; ++i) tau += A[i][k] * A[i][j];
            tau /= A1[k];
            for (int i = k; i < nr; ++i) A[i][j] -= tau * A[i][k];
        }
    }
    for (int j = 0; j < nc; ++j) {
        double tau = 0;
        for (int i = j; i < nr; ++i) tau += A[i][j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; ++i) b[i] -= tau * A[i][j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; --i) {
        double sum = 0;
        for (int j = i + 1; j < nc; ++j) sum += A[i][j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

double null_w(int i, int j) { return (double)(((i * 7 + j * 13 + i * j * 5 + 3) % 17) - 8) / 8.0; }

// the canonical null-space basis of the spec (pnp_ref.canonicalize_null_space)
void canonicalize(std::vector<double>& ut, int k) {
    std::vector<double> V(12 * k), WV(k * k, 0.0), B(12 * k, 0.0);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < 12; ++r) V[r * k + c] = ut[(11 - c) * 12 + r];
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j)
            for (int r = 0; r < 12; ++r) WV[i * k + j] += null_w(r, i) * V[r * k + j];
    // inverse by Gauss-Jordan with partial pivoting
    std::vector<double> G(k * 2 * k, 0.0);
    for (int i = 0; i < k; ++i) {
        for (int j = 0; j < k; ++j) G[i * 2 * k + j] = WV[i * k + j];
        G[i * 2 * k + k + i] = 1.0;
    }
    for (int c = 0; c < k; ++c) {
        int p = c;
        for (int r = c + 1; r < k; ++r)
            if (std::fabs(G[r * 2 * k + c]) > std::fabs(G[p * 2 * k + c])) p = r;
        if (G[p * 2 * k + c] == 0.0) return;
        for (int j = 0; j < 2 * k; ++j) std::swap(G[c * 2 * k + j], G[p * 2 * k + j]);
        const double d = G[c * 2 * k + c];
        for (int j = 0; j < 2 * k; ++j) G[c * 2 * k + j] /= d;
        for (int r = 0; r < k; ++r)
            if (r != c) {
                const double f = G[r * 2 * k + c];
                for (int j = 0; j < 2 * k; ++j) G[r * 2 * k + j] -= f * G[c * 2 * k + j];
            }
    }
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < k; ++c)
            for (int j = 0; j < k; ++j) B[r * k + c] += V[r * k + j] * G[j * 2 * k + k + c];
    for (int c = 0; c < k; ++c) {
        for (int j = 0; j < c; ++j) {
            double d = 0;
            for (int r = 0; r < 12; ++r) d += B[r * k + j] * B[r * k + c];
            for (int r = 0; r < 12; ++r) B[r * k + c] -= d * B[r * k + j];
        }
        double nn = 0;
        for (int r = 0; r < 12; ++r) nn += B[r * k + c] * B[r * k + c];
        nn = std::sqrt(nn);
        for (int r = 0; r < 12; ++r) B[r * k + c] /= nn;
    }
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < 12; ++r) ut[(11 - c) * 12 + r] = B[r * k + c];
}

struct Pose {
    double R[9], t[3], err;
};

// PnPsolver::compute_pose (:523-580) over pws[n][3], us[n][2]
Pose compute_pose(const std::vector<double>& pws, const std::vector<double>& us, const double* cam) {
    const double fu = cam[0], fv = cam[1], uc = cam[2], vc = cam[3];
    const int n = (int)(us.size() / 2);
    double cws[4][3] = {};
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) cws[0][j] += pws[3 * i + j];
    for (int j = 0; j < 3; ++j) cws[0][j] /= n;
    std::vector<double> dtd(9, 0.0), dc, uct;
    for (int i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) dtd[a * 3 + b] += (pws[3 * i + a] - cws[0][a]) * (pws[3 * i + b] - cws[0][b]);
    sym_eig_desc(dtd, 3, dc, uct);
    for (int i = 0; i < 3; ++i) {
        int m = 0;
        for (int j = 1; j < 3; ++j)
            if (std::fabs(uct[3 * i + j]) > std::fabs(uct[3 * i + m])) m = j;
        if (uct[3 * i + m] < 0)
            for (int j = 0; j < 3; ++j) uct[3 * i + j] = -uct[3 * i + j];
    }
    for (int i = 1; i < 4; ++i)
        for (int j = 0; j < 3; ++j) cws[i][j] = cws[0][j] + std::sqrt(dc[i - 1] / n) * uct[3 * (i - 1) + j];
    // ci = pinv(cc), cc[r][c] = cws[c+1][r] - cws[0][r]
    double ci[9];
    {
        std::vector<double> cc(9), s, v;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) cc[r * 3 + c] = cws[c + 1][r] - cws[0][r];
        std::vector<double> a = cc;
        svd_jacobi(a, 3, 3, s, v);
        const double smax = std::max(s[0], std::max(s[1], s[2]));
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double acc = 0;
                for (int j = 0; j < 3; ++j)
                    if (s[j] > 1e-15 * smax) acc += v[r * 3 + j] * a[c * 3 + j] / (s[j] * s[j]);
                ci[r * 3 + c] = acc;
            }
    }
    std::vector<double> alphas(4 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        double d[3];
        for (int j = 0; j < 3; ++j) d[j] = pws[3 * i + j] - cws[0][j];
        for (int j = 0; j < 3; ++j) alphas[4 * i + 1 + j] = d[0] * ci[3 * j] + d[1] * ci[3 * j + 1] + d[2] * ci[3 * j + 2];
        alphas[4 * i] = 1.0 - alphas[4 * i + 1] - alphas[4 * i + 2] - alphas[4 * i + 3];
    }
    // M^T M (fill_M :483-497)
    std::vector<double> mtm(144, 0.0), w12, ut;
    for (int i = 0; i < n; ++i) {
        double r0[12] = {}, r1[12] = {};
        for (int k = 0; k < 4; ++k) {
            const double a = alphas[4 * i + k];
            r0[3 * k] = a * fu;
            r0[3 * k + 2] = a * (uc - us[2 * i]);
            r1[3 * k + 1] = a * fv;
            r1[3 * k + 2] = a * (vc - us[2 * i + 1]);
        }
        for (int a = 0; a < 12; ++a)
            for (int b = 0; b < 12; ++b) mtm[a * 12 + b] += r0[a] * r0[b] + r1[a] * r1[b];
    }
    sym_eig_desc(mtm, 12, w12, ut);
    if (12 - 2 * n > 0) canonicalize(ut, std::min(4, 12 - 2 * n));
    // L_6x10, rho
    const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    double L[6][10], rho[6];
    for (int j = 0; j < 6; ++j) {
        double D[4][3];
        for (int i = 0; i < 4; ++i)
            for (int c = 0; c < 3; ++c) D[i][c] = ut[(11 - i) * 12 + 3 * pa[j] + c] - ut[(11 - i) * 12 + 3 * pb[j] + c];
        auto dot = [&](int x, int y) { return D[x][0] * D[y][0] + D[x][1] * D[y][1] + D[x][2] * D[y][2]; };
        const double row[10] = {dot(0, 0), 2 * dot(0, 1), dot(1, 1), 2 * dot(0, 2), 2 * dot(1, 2),
                                dot(2, 2), 2 * dot(0, 3), 2 * dot(1, 3), 2 * dot(2, 3), dot(3, 3)};
        std::memcpy(L[j], row, sizeof(row));
        rho[j] = 0;
        for (int c = 0; c < 3; ++c) rho[j] += (cws[pa[j]][c] - cws[pb[j]][c]) * (cws[pa[j]][c] - cws[pb[j]][c]);
    }
    auto gauss_newton = [&](double* B) {
        double X[4] = {0, 0, 0, 0};  // gauss_newton's x: kept by a singular qr_solve
        for (int it = 0; it < 5; ++it) {
            double A[6][4], bb[6];
            for (int i = 0; i < 6; ++i) {
                const double* r = L[i];
                A[i][0] = 2 * r[0] * B[0] + r[1] * B[1] + r[3] * B[2] + r[6] * B[3];
                A[i][1] = r[1] * B[0] + 2 * r[2] * B[1] + r[4] * B[2] + r[7] * B[3];
                A[i][2] = r[3] * B[0] + r[4] * B[1] + 2 * r[5] * B[2] + r[8] * B[3];
                A[i][3] = r[6] * B[0] + r[7] * B[1] + r[8] * B[2] + 2 * r[9] * B[3];
                bb[i] = rho[i] - (r[0] * B[0] * B[0] + r[1] * B[0] * B[1] + r[2] * B[1] * B[1] + r[3] * B[0] * B[2] +
                                  r[4] * B[1] * B[2] + r[5] * B[2] * B[2] + r[6] * B[0] * B[3] + r[7] * B[1] * B[3] +
                                  r[8] * B[2] * B[3] + r[9] * B[3] * B[3]);
            }
            qr_solve(A, bb, X);
            for (int k = 0; k < 4; ++k) B[k] += X[k];
        }
    };
    auto r_and_t = [&](const double* B) {
        Pose P;
        double ccs[4][3] = {};
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int c = 0; c < 3; ++c) ccs[j][c] += B[i] * ut[(11 - i) * 12 + 3 * j + c];
        std::vector<double> pcs(3 * (size_t)n);
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) {
                double acc = 0;
                for (int j = 0; j < 4; ++j) acc += alphas[4 * i + j] * ccs[j][c];
                pcs[3 * i + c] = acc;
            }
        if (pcs[2] < 0)
            for (double& x : pcs) x = -x;
        double pc0[3] = {}, pw0[3] = {};
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) {
                pc0[c] += pcs[3 * i + c];
                pw0[c] += pws[3 * i + c];
            }
        for (int c = 0; c < 3; ++c) {
            pc0[c] /= n;
            pw0[c] /= n;
        }
        std::vector<double> abt(9, 0.0), s, v;
        for (int i = 0; i < n; ++i)
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) abt[a * 3 + b] += (pcs[3 * i + a] - pc0[a]) * (pws[3 * i + b] - pw0[b]);
        svd_jacobi(abt, 3, 3, s, v);  // abt columns = U_j s_j
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double acc = 0;
                for (int j = 0; j < 3; ++j) acc += (s[j] > 0 ? abt[r * 3 + j] / s[j] : 0.0) * v[c * 3 + j];
                P.R[r * 3 + c] = acc;
            }
        double* R = P.R;
        const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                           R[2] * (R[3] * R[7] - R[4] * R[6]);
        if (det < 0)
            for (int c = 0; c < 3; ++c) R[6 + c] = -R[6 + c];
        for (int r = 0; r < 3; ++r) P.t[r] = pc0[r] - (R[3 * r] * pw0[0] + R[3 * r + 1] * pw0[1] + R[3 * r + 2] * pw0[2]);
        double e = 0;
        for (int i = 0; i < n; ++i) {
            const double* X = &pws[3 * i];
            const double xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + P.t[0];
            const double yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + P.t[1];
            const double zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + P.t[2];
            const double ue = uc + fu * xc / zc, ve = vc + fv * yc / zc;
            e += std::sqrt((us[2 * i] - ue) * (us[2 * i] - ue) + (us[2 * i + 1] - ve) * (us[2 * i + 1] - ve));
        }
        P.err = e / n;
        return P;
    };
    Pose sols[3];
    const double eps = 2.220446049250313e-16;
    {  // find_betas_approx_1 (:747-781)
        std::vector<double> A(24);
        for (int i = 0; i < 6; ++i) {
            A[4 * i] = L[i][0];
            A[4 * i + 1] = L[i][1];
            A[4 * i + 2] = L[i][3];
            A[4 * i + 3] = L[i][6];
        }
        const std::vector<double> b4 = lstsq(A, 6, 4, rho, eps * 6);
        double B[4];
        if (b4[0] < 0) {
            B[0] = std::sqrt(-b4[0]);
            for (int k = 1; k < 4; ++k) B[k] = -b4[k] / B[0];
        } else {
            B[0] = std::sqrt(b4[0]);
            for (int k = 1; k < 4; ++k) B[k] = b4[k] / B[0];
        }
        gauss_newton(B);
        sols[0] = r_and_t(B);
    }
    for (int ap = 1; ap < 3; ++ap) {  // find_betas_approx_2 (:783-815) / _3 (:817-851)
        const int k = ap == 1 ? 3 : 5;
        std::vector<double> A(6 * k);
        for (int i = 0; i < 6; ++i)
            for (int c = 0; c < k; ++c) A[k * i + c] = L[i][c];
        const std::vector<double> bx = lstsq(A, 6, k, rho, eps * 6);
        double B[4] = {0, 0, 0, 0};
        if (bx[0] < 0) {
            B[0] = std::sqrt(-bx[0]);
            B[1] = bx[2] < 0 ? std::sqrt(-bx[2]) : 0.0;
        } else {
            B[0] = std::sqrt(bx[0]);
            B[1] = bx[2] > 0 ? std::sqrt(bx[2]) : 0.0;
        }
        if (bx[1] < 0) B[0] = -B[0];
        if (ap == 2) B[2] = bx[3] / B[0];
        gauss_newton(B);
        sols[ap] = r_and_t(B);
    }
    int best = 0;
    if (sols[1].err < sols[0].err) best = 1;
    if (sols[2].err < sols[best].err) best = 2;
    return sols[best];
}

// PnPsolver::CheckInliers (:352-386)
int check_inliers(const Pose& P, const float* P3, const float* P2, const float* maxerr, int n, const double* cam,
                  unsigned char* mask) {
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        const double x = P3[3 * i], y = P3[3 * i + 1], z = P3[3 * i + 2];
        const float Xc = (float)(P.R[0] * x + P.R[1] * y + P.R[2] * z + P.t[0]);
        const float Yc = (float)(P.R[3] * x + P.R[4] * y + P.R[5] * z + P.t[1]);
        const float invZc = (float)(1 / (P.R[6] * x + P.R[7] * y + P.R[8] * z + P.t[2]));
        const double ue = cam[2] + cam[0] * (double)Xc * (double)invZc;
        const double ve = cam[3] + cam[1] * (double)Yc * (double)invZc;
        const float dx = (float)((double)P2[2 * i] - ue), dy = (float)((double)P2[2 * i + 1] - ve);
        const bool in = dx * dx + dy * dy < maxerr[i];
        mask[i] = in;
        cnt += in;
    }
    return cnt;
}

}  // namespace

extern "C" {

// The loop body of PnPsolver::iterate (:224-299) over samples[n_samples][4],
// with Refine (:303-349); pnp_ref.ransac_call.  out_int: found, consumed,
// best_inliers, best_hyp, refined_inliers; out_pose: best R (9) t (3),
// refined R (9) t (3).
void orbref_pnp_ransac_call(const float* P3, const float* P2, const float* maxerr, int n, const double* cam,
                            int min_inliers, int best_inliers, const int* samples, int n_samples, int* out_int,
                            double* out_pose) {
    std::vector<unsigned char> mask(n), bmask(n, 0), rmask(n);
    int best = best_inliers, best_hyp = -1, found = 0, consumed = n_samples, refined = 0;
    bool tried = false;
    Pose bP{}, rP{};
    for (int h = 0; h < n_samples; ++h) {
        std::vector<double> pw(12), us(8);
        for (int k = 0; k < 4; ++k) {
            const int i = samples[4 * h + k];
            for (int c = 0; c < 3; ++c) pw[3 * k + c] = P3[3 * i + c];
            us[2 * k] = P2[2 * i];
            us[2 * k + 1] = P2[2 * i + 1];
        }
        const Pose P = compute_pose(pw, us, cam);
        const int c = check_inliers(P, P3, P2, maxerr, n, cam, mask.data());
        if (c < min_inliers) continue;
        if (c > best) {
            best = c;
            best_hyp = h;
            bmask = mask;
            bP = P;
            tried = false;
        }
        if (!tried) {
            std::vector<double> pws, uss;
            for (int i = 0; i < n; ++i)
                if (bmask[i]) {
                    for (int cc = 0; cc < 3; ++cc) pws.push_back(P3[3 * i + cc]);
                    uss.push_back(P2[2 * i]);
                    uss.push_back(P2[2 * i + 1]);
                }
            rP = compute_pose(pws, uss, cam);
            refined = check_inliers(rP, P3, P2, maxerr, n, cam, rmask.data());
            tried = true;
            if (refined > min_inliers) {
                found = 1;
                consumed = h + 1;
                break;
            }
        }
    }
    out_int[0] = found;
    out_int[1] = consumed;
    out_int[2] = best;
    out_int[3] = best_hyp;
    out_int[4] = found ? refined : 0;
    std::memcpy(out_pose, bP.R, 9 * sizeof(double));
    std::memcpy(out_pose + 9, bP.t, 3 * sizeof(double));
    std::memcpy(out_pose + 12, rP.R, 9 * sizeof(double));
    std::memcpy(out_pose + 21, rP.t, 3 * sizeof(double));
}

}  // extern "C"

// qr_solve on its own (tests: the eta-scan case, tests/test_pnp.py)
extern "C" void orbref_qr_solve_6x4(const double* A, const double* b, double* X) {
    double a[6][4], bb[6];
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 4; ++j) a[i][j] = A[i * 4 + j];
        bb[i] = b[i];
    }
    qr_solve(a, bb, X);
}
