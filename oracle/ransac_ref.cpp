/*
 * ransac_ref.cpp -- CPU restatement of the RANSAC inner loops (TEST
 * INFRASTRUCTURE ONLY: the parity oracle for csrc/sim3.hip; the product never
 * links it).
 *
 * Citations: S = /root/reference/ORB-SLAM2/src/Sim3Solver.cpp,
 *            D = /root/reference/ORB-SLAM2/Thirdparty/DBoW2/DUtils/Random.cpp.
 *
 * PARITY STATUS: the reference computes with cv::Mat (OpenCV 2.4: gemm,
 * eigen, Rodrigues), which cannot be built here; this restatement follows
 * the same expressions in float with double accumulation where OpenCV's
 * small-matrix kernels accumulate in double.  GPU vs oracle is compared to
 * a stated tolerance (tests/test_ransac.py); vs OpenCV it is unpinned.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orbref.h"

namespace {

struct Sim3 {
    float R[9], s, t[3];   // rotation, scale, translation (T12 = [sR | t])
    float sR[9];
    float sRi[9], ti[3];   // T21
};

// Symmetric 4x4 eigen-decomposition by the classical Jacobi method with the
// largest off-diagonal pivot (as OpenCV's cv::eigen -> Jacobi does for a
// symmetric float matrix); returns the unit eigenvector of the largest
// eigenvalue.
void eig4_largest(const float N[16], double out[4]) {
    double A[4][4], V[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            A[i][j] = N[4 * i + j];
            V[i][j] = (i == j);
        }
    for (int it = 0; it < 200; ++it) {
        int p = 0, q = 1;
        double mx = 0.0;
        for (int i = 0; i < 4; ++i)
            for (int j = i + 1; j < 4; ++j)
                if (std::fabs(A[i][j]) > mx) { mx = std::fabs(A[i][j]); p = i; q = j; }
        double scale = 0.0;
        for (int i = 0; i < 4; ++i) scale += std::fabs(A[i][i]);
        if (mx <= 1e-17 * (scale + 1e-300)) break;
        const double tau = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
        const double t = (tau >= 0 ? 1.0 : -1.0) / (std::fabs(tau) + std::sqrt(1.0 + tau * tau));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = t * c;
        for (int k = 0; k < 4; ++k) {
            const double akp = A[k][p], akq = A[k][q];
            A[k][p] = c * akp - s * akq;
            A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 4; ++k) {
            const double apk = A[p][k], aqk = A[q][k];
            A[p][k] = c * apk - s * aqk;
            A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 4; ++k) {
            const double vkp = V[k][p], vkq = V[k][q];
            V[k][p] = c * vkp - s * vkq;
            V[k][q] = s * vkp + c * vkq;
        }
    }
    int b = 0;
    for (int i = 1; i < 4; ++i)
        if (A[i][i] > A[b][b]) b = i;
    for (int k = 0; k < 4; ++k) out[k] = V[k][b];
}

// float 3x3 * float 3-vector with double accumulation
float dotd(const float* a, const float* x) {
    double r = 0.0;
    for (int k = 0; k < 3; ++k) r += (double)a[k] * (double)x[k];
    return (float)r;
}

// Sim3Solver::ComputeSim3 (S:225-327); p1[k], p2[k] = point k
Sim3 compute_sim3(const float p1[3][3], const float p2[3][3], bool fix_scale) {
    Sim3 H;
    float O1[3], O2[3], r1[3][3], r2[3][3];
    for (int i = 0; i < 3; ++i) {  // ComputeCentroid (S:213-222)
        O1[i] = (p1[0][i] + p1[1][i] + p1[2][i]) * (1.0f / 3.0f);
        O2[i] = (p2[0][i] + p2[1][i] + p2[2][i]) * (1.0f / 3.0f);
        for (int k = 0; k < 3; ++k) {
            r1[k][i] = p1[k][i] - O1[i];
            r2[k][i] = p2[k][i] - O2[i];
        }
    }
    float M[3][3];  // Pr2 * Pr1^T (S:245)
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 3; ++k) acc += (double)r2[k][i] * (double)r1[k][j];
            M[i][j] = (float)acc;
        }
    // the quaternion matrix N (S:249-273)
    const float N[16] = {M[0][0] + M[1][1] + M[2][2], M[1][2] - M[2][1], M[2][0] - M[0][2], M[0][1] - M[1][0],
                         M[1][2] - M[2][1], M[0][0] - M[1][1] - M[2][2], M[0][1] + M[1][0], M[2][0] + M[0][2],
                         M[2][0] - M[0][2], M[0][1] + M[1][0], -M[0][0] + M[1][1] - M[2][2], M[1][2] + M[2][1],
                         M[0][1] - M[1][0], M[2][0] + M[0][2], M[1][2] + M[2][1], -M[0][0] - M[1][1] + M[2][2]};
    double q[4];
    eig4_largest(N, q);
    const float e[4] = {(float)q[0], (float)q[1], (float)q[2], (float)q[3]};
    // rotation vector 2*atan2(|v|, w) * v/|v| (S:279-287), then Rodrigues
    const double nv = std::sqrt((double)e[1] * e[1] + (double)e[2] * e[2] + (double)e[3] * e[3]);
    const double ang = std::atan2(nv, (double)e[0]);
    double r[3];
    for (int i = 0; i < 3; ++i) r[i] = (float)((double)(float)(2.0 * ang * e[i + 1]) / nv);
    const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < 2.220446049250313e-16) {
        for (int k = 0; k < 9; ++k) H.R[k] = (k % 4 == 0) ? 1.f : 0.f;
    } else {
        const double c = std::cos(th), s = std::sin(th), c1 = 1.0 - c;
        const double x = r[0] / th, y = r[1] / th, z = r[2] / th;
        const double Rd[9] = {c + c1 * x * x,     c1 * x * y - s * z, c1 * x * z + s * y,
                              c1 * x * y + s * z, c + c1 * y * y,     c1 * y * z - s * x,
                              c1 * x * z - s * y, c1 * y * z + s * x, c + c1 * z * z};
        for (int k = 0; k < 9; ++k) H.R[k] = (float)Rd[k];
    }
    float P3[3][3];  // R * Pr2 (S:292)
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) P3[k][i] = dotd(&H.R[3 * i], r2[k]);
    if (!fix_scale) {  // S:295-311
        double nom = 0.0, den = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) {
                nom += (double)r1[k][i] * (double)P3[k][i];
                den += (double)(P3[k][i] * P3[k][i]);
            }
        H.s = (float)(nom / den);
    } else {
        H.s = 1.0f;
    }
    for (int i = 0; i < 3; ++i) {  // t = O1 - s R O2 (S:316)
        double acc = 0.0;
        for (int k = 0; k < 3; ++k) acc += (double)H.R[3 * i + k] * (double)O2[k];
        H.t[i] = O1[i] - (float)(H.s * acc);
    }
    for (int k = 0; k < 9; ++k) H.sR[k] = (float)((double)H.s * H.R[k]);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) H.sRi[3 * i + j] = (float)((1.0 / H.s) * H.R[3 * j + i]);
    for (int i = 0; i < 3; ++i) H.ti[i] = -dotd(&H.sRi[3 * i], H.t);
    return H;
}

void cam_to_image(const float* K, const float* X, float* uv) {  // FromCameraToImage (S:402-420)
    const float invz = 1.0f / X[2];
    uv[0] = K[0] * (X[0] * invz) + K[2];
    uv[1] = K[1] * (X[1] * invz) + K[3];
}

void project(const float* sR, const float* t, const float* K, const float* X, float* uv) {  // Project (S:378-400)
    const float P[3] = {dotd(sR, X) + t[0], dotd(sR + 3, X) + t[1], dotd(sR + 6, X) + t[2]};
    cam_to_image(K, P, uv);
}

// CheckInliers (S:331-358)
int check_inliers(const Sim3& H, int n, const float* X1, const float* X2, const float* e1, const float* e2,
                  const float* K1, const float* K2, uint8_t* mask) {
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        float p1[2], p2[2], q1[2], q2[2];
        cam_to_image(K1, X1 + 3 * i, p1);
        cam_to_image(K2, X2 + 3 * i, p2);
        project(H.sR, H.t, K1, X2 + 3 * i, q1);
        project(H.sRi, H.ti, K2, X1 + 3 * i, q2);
        const float a0 = p1[0] - q1[0], a1 = p1[1] - q1[1], b0 = q2[0] - p2[0], b1 = q2[1] - p2[1];
        const float err1 = (float)((double)a0 * a0 + (double)a1 * a1);
        const float err2 = (float)((double)b0 * b0 + (double)b1 * b1);
        const bool in = err1 < e1[i] && err2 < e2[i];
        if (mask) mask[i] = in;
        cnt += in;
    }
    return cnt;
}

}  // namespace

extern "C" {

int orbref_sim3_ransac(int n, const float* X1, const float* X2, const float* maxerr1, const float* maxerr2,
                       const float* K1, const float* K2, int fix_scale, int min_inliers, int best_inliers, int n_hyp,
                       const int* samples, int* out_ints, float* out_T12, float* out_R12, float* out_t12,
                       float* out_s12, uint8_t* inliers) {
    // Sim3Solver::iterate (S:147-221) over the given triplets
    int best = best_inliers, best_hyp = -1, found = 0, consumed = n_hyp;
    Sim3 B{};
    for (int h = 0; h < n_hyp; ++h) {
        float p1[3][3], p2[3][3];
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 3; ++i) {
                p1[k][i] = X1[3 * samples[3 * h + k] + i];
                p2[k][i] = X2[3 * samples[3 * h + k] + i];
            }
        const Sim3 H = compute_sim3(p1, p2, fix_scale != 0);
        const int c = check_inliers(H, n, X1, X2, maxerr1, maxerr2, K1, K2, nullptr);
        if (c >= best) {
            best = c;
            best_hyp = h;
            B = H;
            if (c > min_inliers) {
                found = 1;
                consumed = h + 1;
                break;
            }
        }
    }
    if (best_hyp >= 0) {
        check_inliers(B, n, X1, X2, maxerr1, maxerr2, K1, K2, inliers);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) out_T12[4 * i + j] = B.sR[3 * i + j];
            out_T12[4 * i + 3] = B.t[i];
            out_t12[i] = B.t[i];
        }
        out_T12[12] = out_T12[13] = out_T12[14] = 0.f;
        out_T12[15] = 1.f;
        std::memcpy(out_R12, B.R, sizeof(B.R));
        *out_s12 = B.s;
    }
    out_ints[0] = found;
    out_ints[1] = consumed;
    out_ints[2] = best;
    out_ints[3] = best_hyp;
    return 0;
}

}  // extern "C"
