// ransac.cpp -- host side of the RANSAC entry points (include/orbgpu_ransac.h):
// the glibc-compatible random stream and the Sim3 / PnP batch drivers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>

#include "../../include/orbgpu_init.h"
#include "../../include/orbgpu_ransac.h"
#include "host_common.h"
#include "host_ctx.h"
#include "ransac_kernels.h"

using namespace orbgpu;

namespace {

// glibc random_r.c, TYPE_3 (x**31 + x**3 + 1), the generator behind rand():
// srandom_r fills r[0..30] with 16807^i * seed mod (2^31 - 1) (Schrage's
// method, seed 0 -> 1), sets front = 3, rear = 0 and discards 310 outputs;
// random_r adds r[rear] into r[front], returns the sum >> 1 and advances
// both indices cyclically.
constexpr int kDeg = 31, kSep = 3;

int32_t next(orbgpu_rand_state* st) {
    uint32_t val = (uint32_t)st->r[st->f] + (uint32_t)st->r[st->b];
    st->r[st->f] = (int32_t)val;
    const int32_t out = (int32_t)(val >> 1);
    if (++st->f >= kDeg) {
        st->f = 0;
        ++st->b;
    } else if (++st->b >= kDeg) {
        st->b = 0;
    }
    return out;
}

void seed(orbgpu_rand_state* st, unsigned int s) {
    if (s == 0) s = 1;
    st->r[0] = (int32_t)s;
    int32_t word = (int32_t)s;
    for (int i = 1; i < kDeg; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        st->r[i] = word;
    }
    st->f = kSep;
    st->b = 0;
    for (int k = 0; k < kDeg * 10; ++k) (void)next(st);
}

std::mutex g_rand_mu;
orbgpu_rand_state g_rand = [] {
    orbgpu_rand_state s;
    seed(&s, 1);  // glibc's initial state equals srand(1)
    return s;
}();

}  // namespace

extern "C" {

void orbgpu_srand_r(orbgpu_rand_state* st, unsigned int s) { seed(st, s); }
int orbgpu_rand_r(orbgpu_rand_state* st) { return next(st); }

void orbgpu_srand(unsigned int s) {
    std::lock_guard<std::mutex> lk(g_rand_mu);
    seed(&g_rand, s);
}

int orbgpu_rand(void) {
    std::lock_guard<std::mutex> lk(g_rand_mu);
    return next(&g_rand);
}

int orbgpu_random_int(int min, int max) {
    const int d = max - min + 1;
    return int(((double)orbgpu_rand() / ((double)2147483647 + 1.0)) * d) + min;
}

void orbgpu_rand_get_state(orbgpu_rand_state* out) {
    std::lock_guard<std::mutex> lk(g_rand_mu);
    *out = g_rand;
}

void orbgpu_rand_set_state(const orbgpu_rand_state* in) {
    std::lock_guard<std::mutex> lk(g_rand_mu);
    g_rand = *in;
}

void orbgpu_seed_rand_once(unsigned int s) {
    static std::atomic<bool> seeded{false};
    bool expect = false;
    if (seeded.compare_exchange_strong(expect, true)) orbgpu_srand(s);
}

int orbgpu_init_draw_sets(int n_matches, int n_iter, int* sets) {
    if (n_matches < 8 || n_iter < 0 || (n_iter > 0 && !sets)) return fail(ORBGPU_ERR_ARG, "invalid argument");
    std::vector<int> avail;
    for (int it = 0; it < n_iter; ++it) {
        avail.resize(n_matches);
        for (int i = 0; i < n_matches; ++i) avail[i] = i;
        for (int j = 0; j < 8; ++j) {
            const int r = orbgpu_random_int(0, (int)avail.size() - 1);
            sets[8 * it + j] = avail[r];
            avail[r] = avail.back();
            avail.pop_back();
        }
    }
    return ORBGPU_OK;
}

size_t orbgpu_sim3_workspace_bytes(int total_samples) {
    return (size_t)(total_samples > 0 ? total_samples : 1) * sim3_hyp_bytes();
}

int orbgpu_sim3_ransac_batch_device(int batch, const orbgpu_sim3_problem* d_problems, int max_hyp,
                                    const float* d_X1, const float* d_X2, const float* d_maxerr1,
                                    const float* d_maxerr2, const int* d_samples, void* d_workspace,
                                    orbgpu_sim3_result* d_results, uint8_t* d_inliers, void* stream) {
    if (batch < 0 || max_hyp < 0 ||
        (batch > 0 && (!d_problems || !d_X1 || !d_X2 || !d_maxerr1 || !d_maxerr2 || !d_samples || !d_workspace ||
                       !d_results || !d_inliers)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_sim3_ransac(batch, d_problems, max_hyp, d_X1, d_X2, d_maxerr1, d_maxerr2, d_samples, d_workspace,
                               d_results, d_inliers, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_sim3_ransac_batch(int batch, const orbgpu_sim3_problem* problems, int total_points, const float* X1,
                             const float* X2, const float* maxerr1, const float* maxerr2, int total_samples,
                             const int* samples, orbgpu_sim3_result* results, uint8_t* inliers) {
    if (batch < 0 || total_points < 0 || total_samples < 0 || (batch > 0 && (!problems || !results)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    for (int b = 0; b < batch; ++b) {  // bounds of every problem against the arrays
        const orbgpu_sim3_problem& p = problems[b];
        if (p.n < 0 || p.offset < 0 || p.offset + p.n > total_points || p.n_hyp < 0 || p.sample_offset < 0 ||
            p.sample_offset + p.n_hyp > total_samples)
            return fail(ORBGPU_ERR_ARG, "problem " + std::to_string(b) + " is out of the array bounds");
        if (p.n_hyp > 0 && p.n < 3) return fail(ORBGPU_ERR_ARG, "a hypothesis needs 3 correspondences");
        for (int h = 0; h < 3 * p.n_hyp; ++h) {
            const int idx = samples[3 * (size_t)p.sample_offset + h];
            if (idx < 0 || idx >= p.n) return fail(ORBGPU_ERR_ARG, "sample index out of range");
        }
    }
    int rc = check_device();
    if (rc) return rc;
    if (batch == 0) return ORBGPU_OK;
    int max_hyp = 0;
    for (int b = 0; b < batch; ++b) max_hyp = std::max(max_hyp, problems[b].n_hyp);
    const size_t np = (size_t)(total_points > 0 ? total_points : 1), ns = (size_t)(total_samples > 0 ? total_samples : 1);
    const size_t tp = (size_t)total_points, ts = (size_t)total_samples;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const orbgpu_sim3_problem* dp;
    const float *dx1, *dx2, *de1, *de2;
    const int* ds;
    orbgpu_sim3_result* dr;
    uint8_t* di;
    void* dw;
    rc = call.run([&](HostCall& A) {
        dp = A.in(problems, (size_t)batch);
        dx1 = A.inout(X1, 3 * tp, 3 * np);
        dx2 = A.inout(X2, 3 * tp, 3 * np);
        de1 = A.inout(maxerr1, tp, np);
        de2 = A.inout(maxerr2, tp, np);
        ds = A.inout(samples, 3 * ts, 3 * ns);
        di = A.inout(inliers, tp, np);
        dr = A.out<orbgpu_sim3_result>((size_t)batch);
        dw = A.out<uint8_t>(orbgpu_sim3_workspace_bytes(total_samples));
    });
    if (rc) return rc;
    rc = orbgpu_sim3_ransac_batch_device(batch, dp, max_hyp, dx1, dx2, de1, de2, ds, dw, dr, di, ctx->stream);
    if (rc) return rc;
    call.fetch(dr, results, sizeof(*dr) * batch);
    call.fetch(di, inliers, tp);
    return call.finish();
}

size_t orbgpu_pnp_workspace_bytes(int total_points, int total_samples) {
    const size_t hyps = (size_t)(total_samples > 0 ? total_samples : 1) * pnp_hyp_bytes();
    return (hyps + 255) / 256 * 256 + (size_t)(total_points > 0 ? total_points : 1) * sizeof(int);
}

int orbgpu_pnp_ransac_batch_device(int batch, const orbgpu_pnp_problem* d_problems, int max_hyp,
                                   int total_points, int total_samples, const float* d_P3w, const float* d_P2,
                                   const float* d_maxerr, const int* d_samples, void* d_workspace,
                                   orbgpu_pnp_result* d_results, uint8_t* d_best_mask, uint8_t* d_refined_mask,
                                   void* stream) {
    if (batch < 0 || max_hyp < 0 || total_points < 0 || total_samples < 0 ||
        (batch > 0 && (!d_problems || !d_P3w || !d_P2 || !d_maxerr || !d_samples || !d_workspace || !d_results ||
                       !d_best_mask || !d_refined_mask)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    int rc = check_device();
    if (rc) return rc;
    const size_t hyps = (size_t)(total_samples > 0 ? total_samples : 1) * pnp_hyp_bytes();
    int* lists = reinterpret_cast<int*>(static_cast<uint8_t*>(d_workspace) + (hyps + 255) / 256 * 256);
    ORB_HIP(launch_pnp_ransac(batch, d_problems, max_hyp, d_P3w, d_P2, d_maxerr, d_samples, d_workspace, lists,
                              d_results, d_best_mask, d_refined_mask, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_pnp_ransac_batch(int batch, const orbgpu_pnp_problem* problems, int total_points, const float* P3w,
                            const float* P2, const float* maxerr, int total_samples, const int* samples,
                            orbgpu_pnp_result* results, uint8_t* best_mask, uint8_t* refined_mask) {
    if (batch < 0 || total_points < 0 || total_samples < 0 || (batch > 0 && (!problems || !results)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    for (int b = 0; b < batch; ++b) {
        const orbgpu_pnp_problem& p = problems[b];
        if (p.n < 0 || p.offset < 0 || p.offset + p.n > total_points || p.n_hyp < 0 || p.sample_offset < 0 ||
            p.sample_offset + p.n_hyp > total_samples)
            return fail(ORBGPU_ERR_ARG, "problem " + std::to_string(b) + " is out of the array bounds");
        if (p.n_hyp > 0 && p.n < 4) return fail(ORBGPU_ERR_ARG, "a hypothesis needs 4 correspondences");
        for (int h = 0; h < 4 * p.n_hyp; ++h) {
            const int idx = samples[4 * (size_t)p.sample_offset + h];
            if (idx < 0 || idx >= p.n) return fail(ORBGPU_ERR_ARG, "sample index out of range");
        }
    }
    int rc = check_device();
    if (rc) return rc;
    if (batch == 0) return ORBGPU_OK;
    int max_hyp = 0;
    for (int b = 0; b < batch; ++b) max_hyp = std::max(max_hyp, problems[b].n_hyp);
    const size_t np = (size_t)(total_points > 0 ? total_points : 1), ns = (size_t)(total_samples > 0 ? total_samples : 1);
    const size_t tp = (size_t)total_points, ts = (size_t)total_samples;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const orbgpu_pnp_problem* dp;
    const float *d3, *d2, *de;
    const int* ds;
    orbgpu_pnp_result* dr;
    uint8_t *dbm, *drm;
    void* dw;
    rc = call.run([&](HostCall& A) {
        dp = A.in(problems, (size_t)batch);
        d3 = A.inout(P3w, 3 * tp, 3 * np);
        d2 = A.inout(P2, 2 * tp, 2 * np);
        de = A.inout(maxerr, tp, np);
        ds = A.inout(samples, 4 * ts, 4 * ns);
        dbm = A.inout(best_mask, tp, np);
        drm = A.inout(refined_mask, tp, np);
        dr = A.out<orbgpu_pnp_result>((size_t)batch);
        dw = A.out<uint8_t>(orbgpu_pnp_workspace_bytes(total_points, total_samples));
    });
    if (rc) return rc;
    rc = orbgpu_pnp_ransac_batch_device(batch, dp, max_hyp, total_points, total_samples, d3, d2, de, ds, dw, dr, dbm,
                                        drm, ctx->stream);
    if (rc) return rc;
    call.fetch(dr, results, sizeof(*dr) * batch);
    call.fetch(dbm, best_mask, tp);
    call.fetch(drm, refined_mask, tp);
    return call.finish();
}

}  // extern "C"
