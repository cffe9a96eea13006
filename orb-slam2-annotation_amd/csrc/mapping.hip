// mapping.hip -- LocalMapping::CreateNewMapPoints' per-match triangulation
// (src/LocalMapping.cpp:369-515, include/orbgpu_mapping.h).
//
// The reference loops over the matched pairs of each neighbour keyframe and
// every pair is independent up to the MapPoint it creates: one thread per
// match, one launch for all neighbours (blockIdx.y = neighbour).  Arithmetic
// follows the reference's float expressions; cv::Mat products of float
// matrices accumulate in double (OpenCV's small gemm), Mat::dot returns a
// double that is added to the float translation before rounding; the 4x4
// SVD is one-sided Jacobi in double (OpenCV's float Jacobi is not
// reproducible bit for bit).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/orbgpu_mapping.h"
#include "epnp.h"
#include "host_common.h"

namespace orbgpu {

namespace {

constexpr int kMapThreads = 128;

// cv::Mat row . x3D (double) + t (float), rounded once
__device__ inline float rowdot_t(const float* T, int r, const float* x) {
    return (float)((double)T[4 * r] * x[0] + (double)T[4 * r + 1] * x[1] + (double)T[4 * r + 2] * x[2] +
                   (double)T[4 * r + 3]);
}

// Rwc * v = Rcw^T v (gemm, double accumulation)
__device__ inline void rwc_mul(const float* T, const float* v, float* out) {
    for (int j = 0; j < 3; ++j)
        out[j] = (float)((double)T[j] * v[0] + (double)T[4 + j] * v[1] + (double)T[8 + j] * v[2]);
}

// cv::norm of a 3x1 CV_32F Mat: the double square root of the double sum
__device__ inline double norm3d(const float* v) {
    return sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2]);
}
// ... assigned to a float (float dist = cv::norm(...))
__device__ inline float norm3f(const float* v) { return (float)norm3d(v); }

// KeyFrame::UnprojectStereo (KeyFrame.cpp:747-775): Twc * (x, y, z) of the raw keypoint
__device__ inline bool unproject_stereo(const orbgpu_mapping_kf& K, int i, float* X) {
    const float z = K.depth[i];
    if (!(z > 0)) return false;
    const float u = K.kps[i].x, v = K.kps[i].y;
    const float xc[3] = {(u - K.cx) * z * K.invfx, (v - K.cy) * z * K.invfy, z};
    float r[3];
    rwc_mul(K.Tcw, xc, r);  // Twc.rowRange(0,3).colRange(0,3) * x3Dc + Twc(0:3, 3), Twc(0:3, 3) = Ow
    for (int j = 0; j < 3; ++j) X[j] = r[j] + K.Ow[j];  // the repo's "R*x + t" convention (proj.hip transform)
    return true;
}

// the reprojection test of one keyframe (:437-487); mbf = the CURRENT keyframe's (the
// reference uses mpCurrentKeyFrame->mbf for both)
__device__ inline bool reproj_ok(const orbgpu_mapping_kf& K, const float* X, const orbgpu_keypoint& kp, float ur,
                                 bool stereo, float mbf, float z) {
    const float sigma2 = K.level_sigma2[kp.octave & 15];
    const float x = rowdot_t(K.Tcw, 0, X), y = rowdot_t(K.Tcw, 1, X);
    const float invz = 1.0f / z;
    const float u = K.fx * x * invz + K.cx, v = K.fy * y * invz + K.cy;
    const float ex = u - kp.x, ey = v - kp.y;
    if (!stereo) return !((double)(ex * ex + ey * ey) > 5.991 * (double)sigma2);
    const float ur_p = u - mbf * invz;
    const float er = ur_p - ur;
    return !((double)(ex * ex + ey * ey + er * er) > 7.8 * (double)sigma2);
}

__global__ __launch_bounds__(kMapThreads) void triangulate_kernel(const orbgpu_mapping_job* __restrict__ jobs) {
    const orbgpu_mapping_job& J = jobs[blockIdx.y];
    const int m = blockIdx.x * kMapThreads + threadIdx.x;
    if (m >= J.n) return;
    const orbgpu_mapping_kf& A = J.kf1;
    const orbgpu_mapping_kf& B = J.kf2;
    const int idx1 = J.pairs[2 * m], idx2 = J.pairs[2 * m + 1];
    float* out = J.x3d + 3 * (size_t)m;
    J.ok[m] = 0;
    out[0] = out[1] = out[2] = 0.f;
    if (idx1 < 0 || idx1 >= A.n || idx2 < 0 || idx2 >= B.n) return;
    const orbgpu_keypoint kp1 = A.kps_un[idx1], kp2 = B.kps_un[idx2];
    const float ur1 = A.u_right ? A.u_right[idx1] : -1.f, ur2 = B.u_right ? B.u_right[idx2] : -1.f;
    const bool st1 = ur1 >= 0, st2 = ur2 >= 0;
    const float xn1[3] = {(kp1.x - A.cx) * A.invfx, (kp1.y - A.cy) * A.invfy, 1.0f};
    const float xn2[3] = {(kp2.x - B.cx) * B.invfx, (kp2.y - B.cy) * B.invfy, 1.0f};
    float ray1[3], ray2[3];
    rwc_mul(A.Tcw, xn1, ray1);
    rwc_mul(B.Tcw, xn2, ray2);
    const double dot = (double)ray1[0] * ray2[0] + (double)ray1[1] * ray2[1] + (double)ray1[2] * ray2[2];
    // ray1.dot(ray2) / (cv::norm(ray1) * cv::norm(ray2)): dot, norms and their
    // product in double, the quotient assigned to the float (LocalMapping.cpp:410)
    const float cosRays = (float)(dot / (norm3d(ray1) * norm3d(ray2)));
    float cosStereo = cosRays + 1;
    float cosStereo1 = cosStereo, cosStereo2 = cosStereo;
    if (st1) cosStereo1 = cosf(2 * atan2f(A.b / 2, A.depth[idx1]));
    else if (st2) cosStereo2 = cosf(2 * atan2f(B.b / 2, B.depth[idx2]));
    cosStereo = fminf(cosStereo1, cosStereo2);
    float X[3];
    if (cosRays < cosStereo && cosRays > 0 && (st1 || st2 || (double)cosRays < 0.9998)) {
        double M[16];  // A.row(0) = xn1(0) * Tcw1.row(2) - Tcw1.row(0), ...
        for (int c = 0; c < 4; ++c) {
            M[c] = (double)(xn1[0] * A.Tcw[8 + c] - A.Tcw[c]);
            M[4 + c] = (double)(xn1[1] * A.Tcw[8 + c] - A.Tcw[4 + c]);
            M[8 + c] = (double)(xn2[0] * B.Tcw[8 + c] - B.Tcw[c]);
            M[12 + c] = (double)(xn2[1] * B.Tcw[8 + c] - B.Tcw[4 + c]);
        }
        double s[4], v[16];
        epnp::svd_hestenes<4, 4>(M, s, v);
        int jmin = 0;
        for (int j = 1; j < 4; ++j)
            if (s[j] < s[jmin]) jmin = j;
        const float w = (float)v[12 + jmin];
        if (w == 0.0f) return;
        for (int k = 0; k < 3; ++k) X[k] = (float)v[4 * k + jmin] / w;
    } else if (st1 && cosStereo1 < cosStereo2) {
        if (!A.depth || !unproject_stereo(A, idx1, X)) return;
    } else if (st2 && cosStereo2 < cosStereo1) {
        if (!B.depth || !unproject_stereo(B, idx2, X)) return;
    } else {
        return;  // no stereo and very low parallax
    }
    const float z1 = rowdot_t(A.Tcw, 2, X);
    if (z1 <= 0) return;
    const float z2 = rowdot_t(B.Tcw, 2, X);
    if (z2 <= 0) return;
    if (!reproj_ok(A, X, kp1, ur1, st1, A.bf, z1)) return;
    if (!reproj_ok(B, X, kp2, ur2, st2, A.bf, z2)) return;
    const float n1[3] = {X[0] - A.Ow[0], X[1] - A.Ow[1], X[2] - A.Ow[2]};
    const float n2[3] = {X[0] - B.Ow[0], X[1] - B.Ow[1], X[2] - B.Ow[2]};
    const float dist1 = norm3f(n1), dist2 = norm3f(n2);
    if (dist1 == 0 || dist2 == 0) return;
    const float ratioDist = dist2 / dist1;
    const float ratioOctave = A.scale_factors[kp1.octave & 15] / B.scale_factors[kp2.octave & 15];
    const float ratioFactor = 1.5f * J.scale_factor;
    if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) return;
    out[0] = X[0];
    out[1] = X[1];
    out[2] = X[2];
    J.ok[m] = 1;
}

}  // namespace

}  // namespace orbgpu

using namespace orbgpu;

extern "C" int orbgpu_triangulate_matches_batch_device(int njobs, const orbgpu_mapping_job* d_jobs, int max_n,
                                                       void* stream) {
    if (njobs < 0 || max_n < 0 || (njobs > 0 && !d_jobs)) return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (njobs == 0 || max_n == 0) return ORBGPU_OK;
    if (njobs > 65535) return fail(ORBGPU_ERR_ARG, "at most 65535 jobs per launch");
    int rc = check_device();
    if (rc) return rc;
    hipLaunchKernelGGL(triangulate_kernel, dim3((max_n + kMapThreads - 1) / kMapThreads, njobs), dim3(kMapThreads), 0,
                       (hipStream_t)stream, d_jobs);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

extern "C" int orbgpu_triangulate_matches(const orbgpu_mapping_job* job) {
    if (!job || job->n < 0 || (job->n > 0 && (!job->pairs || !job->x3d || !job->ok)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    const orbgpu_mapping_kf* ks[2] = {&job->kf1, &job->kf2};
    for (const orbgpu_mapping_kf* k : ks)
        if (k->n < 0 || (k->n > 0 && (!k->kps_un || !k->kps)) || (k->u_right && !k->depth))
            return fail(ORBGPU_ERR_ARG, "keyframe arrays missing (u_right needs depth)");
    if (job->n == 0) return ORBGPU_OK;
    int rc = check_device();
    if (rc) return rc;
    std::vector<void*> allocs;
    bool ok = true;
    auto up = [&](const void* src, size_t bytes) -> void* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 4)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        allocs.push_back(d);
        if (src && bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
        return d;
    };
    orbgpu_mapping_job d = *job;
    orbgpu_mapping_kf* dk[2] = {&d.kf1, &d.kf2};
    for (int i = 0; i < 2; ++i) {
        const orbgpu_mapping_kf& s = *ks[i];
        dk[i]->kps_un = (const orbgpu_keypoint*)up(s.kps_un, sizeof(orbgpu_keypoint) * (size_t)s.n);
        dk[i]->kps = (const orbgpu_keypoint*)up(s.kps, sizeof(orbgpu_keypoint) * (size_t)s.n);
        dk[i]->u_right = s.u_right ? (const float*)up(s.u_right, 4 * (size_t)s.n) : nullptr;
        dk[i]->depth = s.depth ? (const float*)up(s.depth, 4 * (size_t)s.n) : nullptr;
    }
    const int n = job->n;
    d.pairs = (const int*)up(job->pairs, 8 * (size_t)n);
    d.x3d = (float*)up(nullptr, 12 * (size_t)n);
    d.ok = (uint8_t*)up(nullptr, (size_t)n);
    orbgpu_mapping_job* dj = (orbgpu_mapping_job*)up(&d, sizeof(d));
    auto cleanup = [&]() {
        for (void* p : allocs) (void)hipFree(p);
    };
    if (!ok) {
        cleanup();
        return fail(ORBGPU_ERR_HIP, "upload failed");
    }
    rc = orbgpu_triangulate_matches_batch_device(1, dj, n, nullptr);
    ok = !rc && hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(job->x3d, d.x3d, 12 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(job->ok, d.ok, (size_t)n, hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (rc) return rc;
    if (!ok) return fail(ORBGPU_ERR_HIP, "triangulation failed");
    return ORBGPU_OK;
}
