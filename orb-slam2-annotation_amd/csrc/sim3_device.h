// sim3_device.h -- Sim3Solver device arithmetic shared by the RANSAC
// kernels (sim3.hip: one iterate() call per solver; loop.hip: LoopClosing's
// round-robin ComputeSim3 over all candidates of a query).
//   compute_sim3  ComputeSim3 (src/Sim3Solver.cpp:225-327): Horn's closed form
//   is_inlier     CheckInliers' per-correspondence test (:331-358, Project
//                 :378-400, FromCameraToImage :402-420)
// Arithmetic follows the reference's cv::Mat expressions: float storage,
// small float matrix products accumulated in double (OpenCV's
// GEMMSingleMul<float,double>), quaternion matrix entries formed in float,
// angle-axis and Rodrigues in double.
#pragma once

#include <hip/hip_runtime.h>

namespace orbgpu {
namespace sim3dev {

struct Hyp {
    float sR[9], t[3];    // T12 = [sR | t]
    float sRi[9], ti[3];  // T21
    float R[9];
    float s;
};

__device__ __forceinline__ float gemv_row(const float* a, const float* x) {  // double-accumulated float dot of 3
    return (float)((double)a[0] * (double)x[0] + (double)a[1] * (double)x[1] + (double)a[2] * (double)x[2]);
}

// cyclic Jacobi on a symmetric 4x4; returns the eigenvector of the largest eigenvalue
__device__ __forceinline__ void dominant_eigvec4(const float Nf[16], double v_out[4]) {
    double a[4][4], v[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            a[i][j] = Nf[i * 4 + j];
            v[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int i = 0; i < 4; ++i) {
            diag += a[i][i] * a[i][i];
            for (int j = i + 1; j < 4; ++j) off += a[i][j] * a[i][j];
        }
        if (off <= 1e-30 * (diag + 1e-300)) break;
        // fully unrolled: every a[][] / v[][] index is a constant, so the
        // matrices stay in registers (a loop over (p, q) put them in scratch)
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                const double apq = a[p][q];
                if (apq == 0.0) continue;
                const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // A <- J^T A J
                    const double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double vkp = v[k][p], vkq = v[k][q];
                    v[k][p] = c * vkp - s * vkq;
                    v[k][q] = s * vkp + c * vkq;
                }
            }
    }
    int best = 0;
    double dbest = a[0][0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (a[i][i] > dbest) {
            best = i;
            dbest = a[i][i];
        }
#pragma unroll
    for (int k = 0; k < 4; ++k) v_out[k] = best == 0 ? v[k][0] : best == 1 ? v[k][1] : best == 2 ? v[k][2] : v[k][3];
}

// ComputeSim3 (Sim3Solver.cpp:225-327); P1[k], P2[k] = point k (xyz)
__device__ __forceinline__ void compute_sim3(const float P1[3][3], const float P2[3][3], bool fix_scale, Hyp& H) {
    float O1[3], O2[3], Pr1[3][3], Pr2[3][3];  // Pr[k][i]: point k, coordinate i
    for (int i = 0; i < 3; ++i) {              // ComputeCentroid :213-222
        O1[i] = (P1[0][i] + P1[1][i] + P1[2][i]) * (1.0f / 3.0f);
        O2[i] = (P2[0][i] + P2[1][i] + P2[2][i]) * (1.0f / 3.0f);
    }
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) {
            Pr1[k][i] = P1[k][i] - O1[i];
            Pr2[k][i] = P2[k][i] - O2[i];
        }
    float M[3][3];  // M = Pr2 * Pr1^T (:245)
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i][j] = (float)((double)Pr2[0][i] * Pr1[0][j] + (double)Pr2[1][i] * Pr1[1][j] +
                              (double)Pr2[2][i] * Pr1[2][j]);
    const float N11 = M[0][0] + M[1][1] + M[2][2], N12 = M[1][2] - M[2][1], N13 = M[2][0] - M[0][2],
                N14 = M[0][1] - M[1][0], N22 = M[0][0] - M[1][1] - M[2][2], N23 = M[0][1] + M[1][0],
                N24 = M[2][0] + M[0][2], N33 = -M[0][0] + M[1][1] - M[2][2], N34 = M[1][2] + M[2][1],
                N44 = -M[0][0] - M[1][1] + M[2][2];
    const float Nm[16] = {N11, N12, N13, N14, N12, N22, N23, N24, N13, N23, N33, N34, N14, N24, N34, N44};
    double q[4];
    dominant_eigvec4(Nm, q);
    const float ev[4] = {(float)q[0], (float)q[1], (float)q[2], (float)q[3]};
    // angle-axis (:283-287): vec = 2*ang*vec/norm(vec)
    const double nv = sqrt((double)ev[1] * ev[1] + (double)ev[2] * ev[2] + (double)ev[3] * ev[3]);
    const double ang = atan2(nv, (double)ev[0]);
    float vec[3];
    for (int i = 0; i < 3; ++i) vec[i] = (float)((double)(float)(2.0 * ang * ev[i + 1]) / nv);
    // cv::Rodrigues (double internally)
    {
        double rx = vec[0], ry = vec[1], rz = vec[2];
        const double theta = sqrt(rx * rx + ry * ry + rz * rz);
        if (theta < 2.220446049250313e-16) {
            for (int k = 0; k < 9; ++k) H.R[k] = (k % 4 == 0) ? 1.f : 0.f;
        } else {
            const double c = cos(theta), s = sin(theta), c1 = 1.0 - c, it = 1.0 / theta;
            rx *= it; ry *= it; rz *= it;
            const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
            const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
            for (int k = 0; k < 9; ++k) H.R[k] = (float)(c * ((k % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[k] + s * rxm[k]);
        }
    }
    float P3[3][3];  // P3 = R * Pr2 (:292)
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) P3[k][i] = gemv_row(&H.R[3 * i], Pr2[k]);
    if (!fix_scale) {  // :295-311
        double nom = 0.0, den = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) {
                nom += (double)Pr1[k][i] * (double)P3[k][i];
                den += (double)(P3[k][i] * P3[k][i]);
            }
        H.s = (float)(nom / den);
    } else {
        H.s = 1.0f;
    }
    // t = O1 - s*R*O2; T12; T21 (:316-327)
    for (int i = 0; i < 3; ++i) {
        const double r = (double)H.R[3 * i] * O2[0] + (double)H.R[3 * i + 1] * O2[1] + (double)H.R[3 * i + 2] * O2[2];
        H.t[i] = O1[i] - (float)(H.s * r);
    }
    for (int k = 0; k < 9; ++k) H.sR[k] = (float)((double)H.s * H.R[k]);
    const double is = 1.0 / H.s;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) H.sRi[3 * i + j] = (float)(is * H.R[3 * j + i]);
    for (int i = 0; i < 3; ++i) H.ti[i] = -gemv_row(&H.sRi[3 * i], H.t);
}

// project a camera-frame point through (Rcw | tcw) and K (Project, :378-400)
__device__ __forceinline__ void project(const float* sR, const float* t, const float* K, const float* X, float& u, float& v) {
    const float px = gemv_row(sR, X) + t[0];
    const float py = gemv_row(sR + 3, X) + t[1];
    const float pz = gemv_row(sR + 6, X) + t[2];
    const float invz = 1.0f / pz;
    const float x = px * invz, y = py * invz;
    u = K[0] * x + K[2];
    v = K[1] * y + K[3];
}

// FromCameraToImage (:402-420)
__device__ __forceinline__ void to_image(const float* K, const float* X, float& u, float& v) {
    const float invz = 1.0f / X[2];
    const float x = X[0] * invz, y = X[1] * invz;
    u = K[0] * x + K[2];
    v = K[1] * y + K[3];
}

__device__ __forceinline__ bool is_inlier(const Hyp& H, const float* K1, const float* K2, const float* X1, const float* X2,
                                 float e1max, float e2max) {
    float u1, v1, u2, v2, pu1, pv1, pu2, pv2;
    to_image(K1, X1, u1, v1);    // mvP1im1
    to_image(K2, X2, u2, v2);    // mvP2im2
    project(H.sR, H.t, K1, X2, pu1, pv1);    // vP2im1 = T12 X2
    project(H.sRi, H.ti, K2, X1, pu2, pv2);  // vP1im2 = T21 X1
    const float d1x = u1 - pu1, d1y = v1 - pv1, d2x = pu2 - u2, d2y = pv2 - v2;
    const float err1 = (float)((double)d1x * d1x + (double)d1y * d1y);
    const float err2 = (float)((double)d2x * d2x + (double)d2y * d2y);
    return err1 < e1max && err2 < e2max;
}

// the same test with the correspondence's own projections mvP1im1 / mvP2im2
// precomputed (the ctor's FromCameraToImage, identical arithmetic)
__device__ __forceinline__ bool is_inlier_pre(const Hyp& H, const float* K1, const float* K2, const float* X1,
                                              const float* X2, float2 p1, float2 p2, float e1max, float e2max) {
    float pu1, pv1, pu2, pv2;
    project(H.sR, H.t, K1, X2, pu1, pv1);    // vP2im1 = T12 X2
    project(H.sRi, H.ti, K2, X1, pu2, pv2);  // vP1im2 = T21 X1
    const float d1x = p1.x - pu1, d1y = p1.y - pv1, d2x = pu2 - p2.x, d2y = pv2 - p2.y;
    const float err1 = (float)((double)d1x * d1x + (double)d1y * d1y);
    const float err2 = (float)((double)d2x * d2x + (double)d2y * d2y);
    return err1 < e1max && err2 < e2max;
}

}  // namespace sim3dev
}  // namespace orbgpu
