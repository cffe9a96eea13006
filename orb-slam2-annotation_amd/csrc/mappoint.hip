// mappoint.hip -- MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cpp:302-380)
// and MapPoint::UpdateNormalAndDepth (:414-457) over batches of points
// (include/orbgpu_mappoint.h).
//
// ComputeDistinctiveDescriptors: one wave per point, lanes on the rows of
// the point's N x N distance matrix (64 rows per pass).  A row's median
// (element (N-1)/2 of its sorted distances, the zero self-distance included)
// is found without storing the row: distances are integers in [0, 256], so
// a 9-step binary search on the value, each step counting the row's
// distances <= the probe, gives the exact order statistic.  The column
// descriptors are wave-uniform (scalar loads); invalid observations (bad
// keyframes) are neither rows nor columns.  The first row with the smallest
// median wins (the reference's strict `<` scan) through a wave minimum of
// (median, index) keys.
//
// UpdateNormalAndDepth: one thread per point, the reference's sequential
// float sum over the observations in map order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/orbgpu_mappoint.h"
#include "host_common.h"

namespace orbgpu {

namespace {

constexpr int kPointWaves = 4;

__device__ inline int hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(64 * kPointWaves) void distinctive_kernel(int n_points, const int* __restrict__ off,
                                                                       const uint8_t* __restrict__ desc,
                                                                       const uint8_t* __restrict__ valid,
                                                                       int* __restrict__ best,
                                                                       int* __restrict__ best_median) {
    const int lane = threadIdx.x & 63;
    const int p = (int)blockIdx.x * kPointWaves + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (p >= n_points) return;
    const int o0 = off[p], n_all = off[p + 1] - o0;
    const uint4* D = reinterpret_cast<const uint4*>(desc) + 2 * (size_t)o0;
    const uint8_t* V = valid ? valid + o0 : nullptr;
    int N = 0;  // vDescriptors.size()
    for (int b = 0; b < n_all; b += 64) {
        const bool v = b + lane < n_all && (!V || V[b + lane]);
        N += __popcll(__ballot(v));
    }
    if (N == 0) {  // no descriptor: mDescriptor stays
        if (lane == 0) {
            best[p] = -1;
            if (best_median) best_median[p] = -1;
        }
        return;
    }
    const int k = (N - 1) >> 1;  // vDists[0.5 * (N - 1)]
    unsigned long long key = ~0ull;
    for (int b = 0; b < n_all; b += 64) {
        const int i = b + lane;
        const bool row = i < n_all && (!V || V[i]);
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
        if (row) {
            a0 = D[2 * i];
            a1 = D[2 * i + 1];
        }
        // smallest m with #{j valid : d(i, j) <= m} > k
        int lo = 0, hi = 256;
        for (int step = 0; step < 9; ++step) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < n_all; ++j) {
                if (V && !V[j]) continue;  // wave-uniform
                cnt += hamming(a0, a1, D[2 * j], D[2 * j + 1]) <= mid ? 1 : 0;
            }
            if (cnt > k) hi = mid;
            else lo = mid + 1;
        }
        if (row) key = min(key, ((unsigned long long)lo << 32) | (unsigned)i);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(key, o, 64);
        key = t < key ? t : key;
    }
    if (lane == 0) {
        best[p] = (int)(key & 0xFFFFFFFFu);
        if (best_median) best_median[p] = (int)(key >> 32);
    }
}

// cv::norm of a float 3-vector: sqrt of the double sum of squares
__device__ inline double norm3(float x, float y, float z) {
    return sqrt(((double)x * x + (double)y * y) + (double)z * z);
}

__global__ __launch_bounds__(256) void normal_depth_kernel(orbgpu_normal_depth_batch b) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= b.n_points) return;
    const int o0 = b.obs_offsets[p], o1 = b.obs_offsets[p + 1];
    if (o1 <= o0) return;  // no observation: the reference returns before writing
    const float px = b.pos[3 * p], py = b.pos[3 * p + 1], pz = b.pos[3 * p + 2];
    float nx = 0.0f, ny = 0.0f, nz = 0.0f;
    for (int o = o0; o < o1; ++o) {
        // normal = normal + normali / cv::norm(normali): cv::scaleAdd(normali, 1/norm, normal)
        const float ax = __fsub_rn(px, b.obs_Ow[3 * o]), ay = __fsub_rn(py, b.obs_Ow[3 * o + 1]),
                    az = __fsub_rn(pz, b.obs_Ow[3 * o + 2]);
        const float s = (float)(1.0 / norm3(ax, ay, az));
        nx = __fadd_rn(__fmul_rn(ax, s), nx);
        ny = __fadd_rn(__fmul_rn(ay, s), ny);
        nz = __fadd_rn(__fmul_rn(az, s), nz);
    }
    const float inv_n = (float)(1.0 / (double)(o1 - o0));  // normal / n: convertTo with scale 1/n
    b.normal[3 * p] = __fmul_rn(nx, inv_n);
    b.normal[3 * p + 1] = __fmul_rn(ny, inv_n);
    b.normal[3 * p + 2] = __fmul_rn(nz, inv_n);
    const float cx = __fsub_rn(px, b.ref_Ow[3 * p]), cy = __fsub_rn(py, b.ref_Ow[3 * p + 1]),
                cz = __fsub_rn(pz, b.ref_Ow[3 * p + 2]);
    const float dist = (float)norm3(cx, cy, cz);
    const float dmax = __fmul_rn(dist, b.ref_level_scale[p]);
    b.max_dist[p] = dmax;
    b.min_dist[p] = __fdiv_rn(dmax, b.ref_max_scale[p]);
}

// host upload helper for the host forms
struct Uploads {
    std::vector<void*> ptrs;
    bool ok = true;
    void* put(const void* src, size_t bytes) {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 16)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        ptrs.push_back(d);
        if (src && bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
        return d;
    }
    ~Uploads() {
        for (void* q : ptrs) (void)hipFree(q);
    }
};

bool check_offsets(int n_points, const int* off) {
    if (off[0] != 0) return false;
    for (int p = 0; p < n_points; ++p)
        if (off[p + 1] < off[p]) return false;
    return true;
}

}  // namespace

}  // namespace orbgpu

using namespace orbgpu;

extern "C" int orbgpu_compute_distinctive_descriptors_batch_device(int n_points, const int* d_obs_offsets,
                                                                   const uint8_t* d_obs_desc,
                                                                   const uint8_t* d_obs_valid, int* d_best,
                                                                   int* d_best_median, void* stream) {
    if (n_points < 0 || (n_points > 0 && (!d_obs_offsets || !d_obs_desc || !d_best)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (n_points == 0) return ORBGPU_OK;
    if ((uintptr_t)d_obs_desc & 15) return fail(ORBGPU_ERR_ARG, "obs_desc must be 16-byte aligned");
    int rc = check_device();
    if (rc) return rc;
    const int blocks = (n_points + kPointWaves - 1) / kPointWaves;
    hipLaunchKernelGGL(distinctive_kernel, dim3(blocks), dim3(64 * kPointWaves), 0, (hipStream_t)stream, n_points,
                       d_obs_offsets, d_obs_desc, d_obs_valid, d_best, d_best_median);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

extern "C" int orbgpu_compute_distinctive_descriptors(int n_points, const int* obs_offsets, const uint8_t* obs_desc,
                                                      const uint8_t* obs_valid, int* best, int* best_median) {
    if (n_points < 0 || (n_points > 0 && (!obs_offsets || !best))) return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (n_points == 0) return ORBGPU_OK;
    if (!check_offsets(n_points, obs_offsets)) return fail(ORBGPU_ERR_ARG, "obs_offsets must start at 0 and not decrease");
    const size_t n_obs = (size_t)obs_offsets[n_points];
    if (n_obs > 0 && !obs_desc) return fail(ORBGPU_ERR_ARG, "obs_desc missing");
    int rc = check_device();
    if (rc) return rc;
    Uploads u;
    const int* d_off = (const int*)u.put(obs_offsets, 4 * ((size_t)n_points + 1));
    const uint8_t* d_desc = (const uint8_t*)u.put(obs_desc, 32 * n_obs);
    const uint8_t* d_valid = obs_valid ? (const uint8_t*)u.put(obs_valid, n_obs) : nullptr;
    int* d_best = (int*)u.put(nullptr, 4 * (size_t)n_points);
    int* d_med = (int*)u.put(nullptr, 4 * (size_t)n_points);
    if (!u.ok) return fail(ORBGPU_ERR_HIP, "upload failed");
    rc = orbgpu_compute_distinctive_descriptors_batch_device(n_points, d_off, d_desc, d_valid, d_best, d_med, nullptr);
    if (rc) return rc;
    ORB_HIP(hipDeviceSynchronize());
    ORB_HIP(hipMemcpy(best, d_best, 4 * (size_t)n_points, hipMemcpyDeviceToHost));
    if (best_median) ORB_HIP(hipMemcpy(best_median, d_med, 4 * (size_t)n_points, hipMemcpyDeviceToHost));
    return ORBGPU_OK;
}

extern "C" int orbgpu_update_normal_and_depth_batch_device(const orbgpu_normal_depth_batch* b, void* stream) {
    if (!b || b->n_points < 0) return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (b->n_points == 0) return ORBGPU_OK;
    if (!b->obs_offsets || !b->pos || !b->ref_Ow || !b->ref_level_scale || !b->ref_max_scale || !b->normal ||
        !b->min_dist || !b->max_dist)
        return fail(ORBGPU_ERR_ARG, "NULL array");
    int rc = check_device();
    if (rc) return rc;
    hipLaunchKernelGGL(normal_depth_kernel, dim3((b->n_points + 255) / 256), dim3(256), 0, (hipStream_t)stream, *b);
    ORB_HIP(hipGetLastError());
    return ORBGPU_OK;
}

extern "C" int orbgpu_update_normal_and_depth(const orbgpu_normal_depth_batch* b) {
    if (!b || b->n_points < 0) return fail(ORBGPU_ERR_ARG, "invalid argument");
    const int n = b->n_points;
    if (n == 0) return ORBGPU_OK;
    if (!b->obs_offsets || !b->pos || !b->ref_Ow || !b->ref_level_scale || !b->ref_max_scale || !b->normal ||
        !b->min_dist || !b->max_dist)
        return fail(ORBGPU_ERR_ARG, "NULL array");
    if (!check_offsets(n, b->obs_offsets)) return fail(ORBGPU_ERR_ARG, "obs_offsets must start at 0 and not decrease");
    const size_t n_obs = (size_t)b->obs_offsets[n];
    if (n_obs > 0 && !b->obs_Ow) return fail(ORBGPU_ERR_ARG, "obs_Ow missing");
    int rc = check_device();
    if (rc) return rc;
    Uploads u;
    orbgpu_normal_depth_batch d = *b;
    d.obs_offsets = (const int*)u.put(b->obs_offsets, 4 * ((size_t)n + 1));
    d.obs_Ow = (const float*)u.put(b->obs_Ow, 12 * n_obs);
    d.pos = (const float*)u.put(b->pos, 12 * (size_t)n);
    d.ref_Ow = (const float*)u.put(b->ref_Ow, 12 * (size_t)n);
    d.ref_level_scale = (const float*)u.put(b->ref_level_scale, 4 * (size_t)n);
    d.ref_max_scale = (const float*)u.put(b->ref_max_scale, 4 * (size_t)n);
    // outputs start from the caller's values (points without observations keep them)
    d.normal = (float*)u.put(b->normal, 12 * (size_t)n);
    d.min_dist = (float*)u.put(b->min_dist, 4 * (size_t)n);
    d.max_dist = (float*)u.put(b->max_dist, 4 * (size_t)n);
    if (!u.ok) return fail(ORBGPU_ERR_HIP, "upload failed");
    rc = orbgpu_update_normal_and_depth_batch_device(&d, nullptr);
    if (rc) return rc;
    ORB_HIP(hipDeviceSynchronize());
    ORB_HIP(hipMemcpy(b->normal, d.normal, 12 * (size_t)n, hipMemcpyDeviceToHost));
    ORB_HIP(hipMemcpy(b->min_dist, d.min_dist, 4 * (size_t)n, hipMemcpyDeviceToHost));
    ORB_HIP(hipMemcpy(b->max_dist, d.max_dist, 4 * (size_t)n, hipMemcpyDeviceToHost));
    return ORBGPU_OK;
}
