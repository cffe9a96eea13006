// proj.cpp -- host side of include/orbgpu_proj.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/orbgpu_proj.h"
#include "host_common.h"
#include "proj_kernels.h"

using namespace orbgpu;

namespace {

struct DeviceArena {  // uploads a call's host arrays; frees them on destruction
    std::vector<void*> ptrs;
    bool ok = true;
    ~DeviceArena() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    const T* up(const T* src, size_t count) {
        if (!src) return nullptr;
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(count * sizeof(T), 4)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        ptrs.push_back(d);
        if (count && hipMemcpy(d, src, count * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) ok = false;
        return static_cast<const T*>(d);
    }
    void* alloc(size_t bytes) {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 4)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        ptrs.push_back(d);
        return d;
    }
};

}  // namespace

extern "C" {

int orbgpu_is_in_frustum_device(const orbgpu_proj_target* target, int n, const float* d_pos, const float* d_normal,
                                const float* d_min_dist, const float* d_max_dist, float viewing_cos_limit,
                                int* d_flags, float* d_track, int* d_track_level, void* stream) {
    if (!target || n < 0 ||
        (n > 0 && (!d_pos || !d_normal || !d_min_dist || !d_max_dist || !d_flags || !d_track || !d_track_level)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (target->n_levels < 1 || target->n_levels > 16) return fail(ORBGPU_ERR_ARG, "n_levels must be 1..16");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_is_in_frustum(*target, n, d_pos, d_normal, d_min_dist, d_max_dist, viewing_cos_limit, d_flags,
                                 d_track, d_track_level, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_search_by_projection_batch_device(int ncalls, const orbgpu_proj_call* d_calls, int stride, int* d_match,
                                             int* d_nmatches, void* stream) {
    if (ncalls < 0 || stride <= 0 || (ncalls > 0 && (!d_calls || !d_match || !d_nmatches)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_search_by_projection(ncalls, d_calls, stride, d_match, d_nmatches, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_search_by_projection(const orbgpu_proj_call* call, int* match, int* nmatches) {
    if (!call || !match || !nmatches) return fail(ORBGPU_ERR_ARG, "NULL argument");
    const orbgpu_proj_call& c = *call;
    if (c.variant < ORBGPU_PROJ_LOCAL || c.variant > ORBGPU_PROJ_KEYFRAME) return fail(ORBGPU_ERR_ARG, "bad variant");
    const int n = c.target.n, m = c.points.n;
    if (n < 0 || m < 0 || n > proj_max_keypoints()) return fail(ORBGPU_ERR_ARG, "target has 0..4096 keypoints");
    if (c.target.n_levels < 1 || c.target.n_levels > 16) return fail(ORBGPU_ERR_ARG, "n_levels must be 1..16");
    if ((n > 0 && (!c.target.kps || !c.target.desc)) || (m > 0 && (!c.points.flags || !c.points.desc)))
        return fail(ORBGPU_ERR_ARG, "missing target/point arrays");
    const bool local = c.variant == ORBGPU_PROJ_LOCAL;
    if (m > 0 && local && (!c.points.track || !c.points.track_level))
        return fail(ORBGPU_ERR_ARG, "LOCAL needs the isInFrustum track fields");
    if (m > 0 && !local && !c.points.pos) return fail(ORBGPU_ERR_ARG, "missing point positions");
    if (m > 0 && (c.variant == ORBGPU_PROJ_SIM3 || c.variant == ORBGPU_PROJ_KEYFRAME) &&
        (!c.points.min_dist || !c.points.max_dist))
        return fail(ORBGPU_ERR_ARG, "missing distance invariance");
    if (m > 0 && c.variant == ORBGPU_PROJ_SIM3 && !c.points.normal) return fail(ORBGPU_ERR_ARG, "missing normals");
    if (m > 0 && c.variant == ORBGPU_PROJ_LAST_FRAME && !c.points.octave) return fail(ORBGPU_ERR_ARG, "missing octaves");
    if (m > 0 && c.check_ori && (c.variant == ORBGPU_PROJ_LAST_FRAME || c.variant == ORBGPU_PROJ_KEYFRAME) &&
        !c.points.angle)
        return fail(ORBGPU_ERR_ARG, "missing source angles");
    if (m > 0 && local) {  // predicted levels index scale_factors
        for (int i = 0; i < m; ++i)
            if ((c.points.flags[i] & ORBGPU_PT_IN_VIEW) &&
                (c.points.track_level[i] < 0 || c.points.track_level[i] >= c.target.n_levels))
                return fail(ORBGPU_ERR_ARG, "track level out of range");
    }
    if (m > 0 && c.variant == ORBGPU_PROJ_LAST_FRAME)
        for (int i = 0; i < m; ++i)
            if (c.points.octave[i] < 0 || c.points.octave[i] >= c.target.n_levels)
                return fail(ORBGPU_ERR_ARG, "source octave out of range");
    int rc = check_device();
    if (rc) return rc;
    DeviceArena A;
    orbgpu_proj_call d = c;
    d.target.kps = A.up(c.target.kps, (size_t)n);
    d.target.desc = A.up(c.target.desc, 32 * (size_t)n);
    d.target.u_right = A.up(c.target.u_right, (size_t)n);
    d.target.occupied = A.up(c.target.occupied, (size_t)n);
    d.points.flags = A.up(c.points.flags, (size_t)m);
    d.points.pos = A.up(c.points.pos, 3 * (size_t)m);
    d.points.normal = A.up(c.points.normal, 3 * (size_t)m);
    d.points.desc = A.up(c.points.desc, 32 * (size_t)m);
    d.points.min_dist = A.up(c.points.min_dist, (size_t)m);
    d.points.max_dist = A.up(c.points.max_dist, (size_t)m);
    d.points.octave = A.up(c.points.octave, (size_t)m);
    d.points.angle = A.up(c.points.angle, (size_t)m);
    d.points.track = A.up(c.points.track, 4 * (size_t)m);
    d.points.track_level = A.up(c.points.track_level, (size_t)m);
    const orbgpu_proj_call* dc = A.up(&d, 1);
    int* dm = static_cast<int*>(A.alloc(4 * (size_t)std::max(n, 1)));
    int* dn = static_cast<int*>(A.alloc(4));
    if (!A.ok) return fail(ORBGPU_ERR_HIP, "upload failed");
    rc = orbgpu_search_by_projection_batch_device(1, dc, std::max(n, 1), dm, dn, nullptr);
    if (rc) return rc;
    if (hipDeviceSynchronize() != hipSuccess ||
        (n && hipMemcpy(match, dm, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) ||
        hipMemcpy(nmatches, dn, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(ORBGPU_ERR_HIP, "SearchByProjection failed");
    return ORBGPU_OK;
}

}  // extern "C"
