// frame.hip -- Frame::UndistortKeyPoints (Frame.cpp:462-496),
// ComputeImageBounds (:498-530) and AssignFeaturesToGrid / PosInGrid
// (:241-259, :434-444) for batches of frames (include/orbgpu_frame.h).
//
// Undistortion restates OpenCV 2.4's cvUndistortPoints as the reference calls
// it (R = identity, P = K): camera and distortion converted to double, five
// fixed-point iterations, the P projection written out with its zero terms so
// every double operation is the one OpenCV performs (no contraction:
// -ffp-contract=off).  One thread per keypoint.
//
// Grid: one 1024-thread block per frame; the (cell << 16 | index) keys of the
// keypoints inside the grid are bitonic-sorted in LDS, which gives every
// cell's indices in increasing order (mGrid's push_back order), then the CSR
// starts come from a scan of the per-cell counts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/orbgpu_frame.h"
#include "host_common.h"

namespace {

constexpr int kCells = ORBGPU_GRID_COLS * ORBGPU_GRID_ROWS;
constexpr int kGridThreads = 1024;
constexpr int kGridKeys = 4096;

struct Cam {
    double fx, fy, cx, cy, k[8];
};

__host__ __device__ inline Cam make_cam(const orbgpu_camera& c) {
    Cam m;
    m.fx = (double)c.fx;
    m.fy = (double)c.fy;
    m.cx = (double)c.cx;
    m.cy = (double)c.cy;
    for (int i = 0; i < 8; ++i) m.k[i] = i < c.ndist ? (double)c.dist[i] : 0.0;
    return m;
}

// cvUndistortPoints for one point (OpenCV 2.4 modules/imgproc/src/undistort.cpp)
__host__ __device__ inline void undistort_point(const Cam& m, float px, float py, float* ox, float* oy) {
    const double ifx = 1. / m.fx, ify = 1. / m.fy;
    double x = ((double)px - m.cx) * ifx;
    double y = ((double)py - m.cy) * ify;
    const double x0 = x, y0 = y;
    const double* k = m.k;
    for (int j = 0; j < 5; ++j) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I = K
    const double xx = m.fx * x + 0.0 * y + m.cx;
    const double yy = 0.0 * x + m.fy * y + m.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

__global__ void undistort_kernel(Cam m, bool distorted, const orbgpu_keypoint* __restrict__ kps,
                                 const int* __restrict__ counts, int cap, orbgpu_keypoint* __restrict__ out) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= counts[b]) return;
    orbgpu_keypoint k = kps[(size_t)b * cap + i];
    if (distorted) undistort_point(m, k.x, k.y, &k.x, &k.y);
    out[(size_t)b * cap + i] = k;
}

__global__ __launch_bounds__(kGridThreads) void grid_kernel(orbgpu_grid_bounds g, const orbgpu_keypoint* __restrict__ kps,
                                                            const int* __restrict__ counts, int cap,
                                                            int* __restrict__ cell_start, int* __restrict__ items) {
    __shared__ uint32_t s_key[kGridKeys];
    __shared__ int s_cnt[kCells + 1];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = counts[b];
    const float invW = (float)ORBGPU_GRID_COLS / (g.max_x - g.min_x);
    const float invH = (float)ORBGPU_GRID_ROWS / (g.max_y - g.min_y);
    for (int c = tid; c <= kCells; c += kGridThreads) s_cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < kGridKeys; i += kGridThreads) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n) {
            const orbgpu_keypoint k = kps[(size_t)b * cap + i];
            const int px = (int)roundf(__fmul_rn(__fsub_rn(k.x, g.min_x), invW));
            const int py = (int)roundf(__fmul_rn(__fsub_rn(k.y, g.min_y), invH));
            if (px >= 0 && px < ORBGPU_GRID_COLS && py >= 0 && py < ORBGPU_GRID_ROWS) {
                const int cell = px * ORBGPU_GRID_ROWS + py;
                key = ((uint32_t)cell << 16) | (uint32_t)i;
                atomicAdd(&s_cnt[cell], 1);
            }
        }
        s_key[i] = key;
    }
    __syncthreads();
    // bitonic sort of kGridKeys keys
    for (int size = 2; size <= kGridKeys; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < kGridKeys / 2; i += kGridThreads) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint32_t a = s_key[lo], c = s_key[hi];
                if ((a > c) == up) {
                    s_key[lo] = c;
                    s_key[hi] = a;
                }
            }
            __syncthreads();
        }
    if (tid == 0) {  // exclusive scan of the 3072 cell counts
        int acc = 0;
        for (int c = 0; c < kCells; ++c) {
            const int v = s_cnt[c];
            s_cnt[c] = acc;
            acc += v;
        }
        s_cnt[kCells] = acc;
    }
    __syncthreads();
    for (int c = tid; c <= kCells; c += kGridThreads) cell_start[(size_t)b * (kCells + 1) + c] = s_cnt[c];
    const int total = s_cnt[kCells];
    for (int i = tid; i < total; i += kGridThreads) items[(size_t)b * cap + i] = (int)(s_key[i] & 0xFFFFu);
}

}  // namespace

extern "C" int orbgpu_compute_image_bounds(const orbgpu_camera* cam, int cols, int rows, orbgpu_grid_bounds* out) {
    if (!cam || !out || cols <= 0 || rows <= 0) return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    if (cam->dist[0] != 0.0f) {
        const Cam m = make_cam(*cam);
        float x[4], y[4];
        const float px[4] = {0.f, (float)cols, 0.f, (float)cols}, py[4] = {0.f, 0.f, (float)rows, (float)rows};
        for (int i = 0; i < 4; ++i) undistort_point(m, px[i], py[i], &x[i], &y[i]);
        out->min_x = std::min(x[0], x[2]);
        out->max_x = std::max(x[1], x[3]);
        out->min_y = std::min(y[0], y[1]);
        out->max_y = std::max(y[2], y[3]);
    } else {
        out->min_x = 0.f;
        out->max_x = (float)cols;
        out->min_y = 0.f;
        out->max_y = (float)rows;
    }
    return ORBGPU_OK;
}

extern "C" int orbgpu_undistort_keypoints_batch_device(const orbgpu_camera* cam, int batch, const orbgpu_keypoint* d_kps,
                                                       const int* d_counts, int kp_capacity, orbgpu_keypoint* d_kps_un,
                                                       void* stream) {
    if (!cam || !d_kps || !d_counts || !d_kps_un || batch < 0 || kp_capacity <= 0 || cam->ndist < 4 || cam->ndist > 5)
        return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    if (batch == 0) return ORBGPU_OK;
    if (int rc = orbgpu::check_device()) return rc;
    (void)hipGetLastError();
    const Cam m = make_cam(*cam);
    hipLaunchKernelGGL(undistort_kernel, dim3((kp_capacity + 255) / 256, batch), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), m, cam->dist[0] != 0.0f, d_kps, d_counts, kp_capacity,
                       d_kps_un);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

extern "C" int orbgpu_assign_features_to_grid_batch_device(int batch, orbgpu_grid_bounds bounds,
                                                           const orbgpu_keypoint* d_kps_un, const int* d_counts,
                                                           int kp_capacity, int* d_cell_start, int* d_cell_items,
                                                           void* stream) {
    if (!d_kps_un || !d_counts || !d_cell_start || !d_cell_items || batch < 0 || kp_capacity <= 0)
        return orbgpu::fail(ORBGPU_ERR_ARG, "invalid argument");
    if (kp_capacity > kGridKeys) return orbgpu::fail(ORBGPU_ERR_UNSUPPORTED, "grid assignment needs kp_capacity <= 4096");
    if (batch == 0) return ORBGPU_OK;
    if (int rc = orbgpu::check_device()) return rc;
    (void)hipGetLastError();
    hipLaunchKernelGGL(grid_kernel, dim3(batch), dim3(kGridThreads), 0, reinterpret_cast<hipStream_t>(stream), bounds,
                       d_kps_un, d_counts, kp_capacity, d_cell_start, d_cell_items);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}
