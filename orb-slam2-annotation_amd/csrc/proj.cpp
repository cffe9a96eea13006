// proj.cpp -- host side of include/orbgpu_proj.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/orbgpu_proj.h"
#include "host_common.h"
#include "host_ctx.h"
#include "proj_kernels.h"

using namespace orbgpu;

namespace {

// the call's host arrays uploaded into A; d = the call with device pointers
void upload_call(HostCall& A, const orbgpu_proj_call& c, orbgpu_proj_call& d) {
    const size_t n = (size_t)c.target.n, m = (size_t)c.points.n;
    d = c;
    d.target.kps = A.in(c.target.kps, n);
    d.target.desc = A.in(c.target.desc, 32 * n);
    d.target.u_right = A.in(c.target.u_right, n);
    d.target.occupied = A.in(c.target.occupied, n);
    d.points.flags = A.in(c.points.flags, m);
    d.points.pos = A.in(c.points.pos, 3 * m);
    d.points.normal = A.in(c.points.normal, 3 * m);
    d.points.desc = A.in(c.points.desc, 32 * m);
    d.points.min_dist = A.in(c.points.min_dist, m);
    d.points.max_dist = A.in(c.points.max_dist, m);
    d.points.octave = A.in(c.points.octave, m);
    d.points.angle = A.in(c.points.angle, m);
    d.points.track = A.in(c.points.track, 4 * m);
    d.points.track_level = A.in(c.points.track_level, m);
}

// argument checks of one host call (orbgpu_search_by_projection)
int check_call(const orbgpu_proj_call& c) {
    if (c.variant < ORBGPU_PROJ_LOCAL || c.variant > ORBGPU_PROJ_SIM3_DIR) return fail(ORBGPU_ERR_ARG, "bad variant");
    const int n = c.target.n, m = c.points.n;
    if (n < 0 || m < 0 || n > proj_max_keypoints()) return fail(ORBGPU_ERR_ARG, "target has 0..4096 keypoints");
    if (c.target.n_levels < 1 || c.target.n_levels > 16) return fail(ORBGPU_ERR_ARG, "n_levels must be 1..16");
    if ((n > 0 && (!c.target.kps || !c.target.desc)) || (m > 0 && (!c.points.flags || !c.points.desc)))
        return fail(ORBGPU_ERR_ARG, "missing target/point arrays");
    const bool local = c.variant == ORBGPU_PROJ_LOCAL;
    if (m > 0 && local && (!c.points.track || !c.points.track_level))
        return fail(ORBGPU_ERR_ARG, "LOCAL needs the isInFrustum track fields");
    if (m > 0 && !local && !c.points.pos) return fail(ORBGPU_ERR_ARG, "missing point positions");
    const bool needs_dist = c.variant == ORBGPU_PROJ_SIM3 || c.variant == ORBGPU_PROJ_KEYFRAME ||
                            c.variant >= ORBGPU_PROJ_FUSE;
    if (m > 0 && needs_dist && (!c.points.min_dist || !c.points.max_dist))
        return fail(ORBGPU_ERR_ARG, "missing distance invariance");
    const bool needs_normal =
        c.variant == ORBGPU_PROJ_SIM3 || c.variant == ORBGPU_PROJ_FUSE || c.variant == ORBGPU_PROJ_FUSE_SIM3;
    if (m > 0 && needs_normal && !c.points.normal) return fail(ORBGPU_ERR_ARG, "missing normals");
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
    return ORBGPU_OK;
}

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
    int rc = check_call(c);
    if (rc) return rc;
    rc = check_device();
    if (rc) return rc;
    // one output entry per target keypoint, or per point for the per-point variants
    const int nout = c.variant >= ORBGPU_PROJ_FUSE ? c.points.n : c.target.n;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall hc(*ctx);
    const orbgpu_proj_call* dc;
    int *dm, *dn;
    rc = hc.run([&](HostCall& A) {
        orbgpu_proj_call d;
        upload_call(A, c, d);
        dc = A.in(&d, 1);
        dm = A.out<int>((size_t)std::max(nout, 1));
        dn = A.out<int>(1);
    });
    if (rc) return rc;
    rc = orbgpu_search_by_projection_batch_device(1, dc, std::max(nout, 1), dm, dn, ctx->stream);
    if (rc) return rc;
    hc.fetch(dm, match, 4 * (size_t)nout);
    hc.fetch(dn, nmatches, 4);
    if ((rc = hc.finish())) return rc;
    if (*nmatches < 0) return fail(ORBGPU_ERR_CAPACITY, "call rejected by the kernel");
    return ORBGPU_OK;
}

int orbgpu_search_by_sim3(const orbgpu_sim3_search* search, int* match12, int* nfound) {
    if (!search || !match12 || !nfound) return fail(ORBGPU_ERR_ARG, "NULL argument");
    const orbgpu_sim3_search& S = *search;
    const int n1 = S.kf1.n, n2 = S.kf2.n;
    if (S.pts1.n != n1 || S.pts2.n != n2)
        return fail(ORBGPU_ERR_ARG, "pts1/pts2 must hold one entry per keypoint of kf1/kf2");
    if (!(S.s12 != 0.0f)) return fail(ORBGPU_ERR_ARG, "s12 must be non-zero");
    // sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(), t21 = -sR21*t12 (ORBmatcher.cpp:1272-1274): scalar
    // products in double rounded to float (cv::MatExpr scaling), t21 accumulated in double (gemm)
    float sR12[9], sR21[9], t21[3];
    const double inv = 1.0 / (double)S.s12;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            sR12[3 * i + j] = (float)((double)S.R12[3 * i + j] * (double)S.s12);
            sR21[3 * i + j] = (float)((double)S.R12[3 * j + i] * inv);
        }
    for (int i = 0; i < 3; ++i)
        t21[i] = -(float)((double)sR21[3 * i] * S.t12[0] + (double)sR21[3 * i + 1] * S.t12[1] +
                          (double)sR21[3 * i + 2] * S.t12[2]);
    orbgpu_proj_call c[2];
    std::memset(c, 0, sizeof(c));
    for (int dir = 0; dir < 2; ++dir) {
        orbgpu_proj_call& k = c[dir];
        k.variant = ORBGPU_PROJ_SIM3_DIR;
        k.th = S.th;
        k.target = dir == 0 ? S.kf2 : S.kf1;
        k.points = dir == 0 ? S.pts1 : S.pts2;
        std::memcpy(k.last_Tcw, dir == 0 ? S.kf1.Tcw : S.kf2.Tcw, sizeof(k.last_Tcw));
        k.target.fx = S.kf1.fx;  // pKF1's intrinsics both ways (:1257-1260)
        k.target.fy = S.kf1.fy;
        k.target.cx = S.kf1.cx;
        k.target.cy = S.kf1.cy;
        k.target.occupied = nullptr;
        const float* R = dir == 0 ? sR21 : sR12;
        const float* t = dir == 0 ? t21 : S.t12;
        for (int i = 0; i < 16; ++i) k.target.Tcw[i] = (i == 15) ? 1.f : 0.f;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) k.target.Tcw[4 * i + j] = R[3 * i + j];
            k.target.Tcw[4 * i + 3] = t[i];
        }
        int rc = check_call(k);
        if (rc) return rc;
    }
    int rc = check_device();
    if (rc) return rc;
    const int stride = std::max(1, std::max(n1, n2));
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const orbgpu_proj_call* dc;
    int *dm, *dn;
    rc = call.run([&](HostCall& A) {
        orbgpu_proj_call d[2];
        upload_call(A, c[0], d[0]);
        upload_call(A, c[1], d[1]);
        dc = A.in(d, 2);
        dm = A.out<int>(2 * (size_t)stride);
        dn = A.out<int>(2);
    });
    if (rc) return rc;
    rc = orbgpu_search_by_projection_batch_device(2, dc, stride, dm, dn, ctx->stream);
    if (rc) return rc;
    std::vector<int> m(2 * (size_t)stride);
    int nn[2];
    call.fetch(dm, m.data(), m.size() * 4);
    call.fetch(dn, nn, 8);
    if ((rc = call.finish())) return rc;
    if (nn[0] < 0 || nn[1] < 0) return fail(ORBGPU_ERR_CAPACITY, "call rejected by the kernel");
    const int* v1 = m.data();            // vnMatch1
    const int* v2 = m.data() + stride;   // vnMatch2
    int found = 0;
    for (int i1 = 0; i1 < n1; ++i1) {    // check agreement (:1472-1488)
        const int idx2 = v1[i1];
        match12[i1] = -1;
        if (idx2 >= 0 && v2[idx2] == i1) {
            match12[i1] = idx2;
            ++found;
        }
    }
    *nfound = found;
    return ORBGPU_OK;
}

}  // extern "C"
