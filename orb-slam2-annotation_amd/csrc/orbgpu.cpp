// orbgpu.cpp -- host driver and C ABI (include/orbgpu.h).
//
// Owns the per-extractor geometry (computed once, with the reference's own
// float arithmetic: ORBextractor.cpp:412-472, :781-795, :545-547, :1127-1128
// and OpenCV-2.4 resize()'s tap tables), the HBM buffers sized for
// max_batch frames, and the launch sequence of one extraction:
//   pyramid level 1..L-1  ->  FAST cells (all levels)  ->  octree (frame x
//   level)  ->  angle + blur + rBRIEF + keypoint fields (one wave per slot).
// Errors raised inside kernels (capacity overflows) are accumulated in a
// device word and reported by orbgpu_extractor_sync(); nothing is silently
// truncated.  There is no CPU fallback: without a gfx950 device every entry
// point fails with ORBGPU_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "../../include/orbgpu_debug.h"
#include "../../include/orbgpu_stereo.h"
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "stereo_kernels.h"
#include "host_common.h"
#include "host_ctx.h"

using namespace orbgpu;

namespace orbgpu {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int check_device() {
    // the arch check once per device and thread (the host-form calls run it on every call)
    static thread_local int checked_dev = -1;
    int dev = 0, n = 0;
    if (checked_dev >= 0 && hipGetDevice(&dev) == hipSuccess && dev == checked_dev) return ORBGPU_OK;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(ORBGPU_ERR_NO_DEVICE, "no HIP device visible");
    ORB_HIP(hipGetDevice(&dev));
    hipDeviceProp_t p;
    ORB_HIP(hipGetDeviceProperties(&p, dev));
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
        return fail(ORBGPU_ERR_NO_DEVICE, std::string("device is ") + p.gcnArchName + ", this build targets gfx950");
    checked_dev = dev;
    return ORBGPU_OK;
}

int validate_device(int device) {
    if (device < 0) return fail(ORBGPU_ERR_ARG, "device ordinal must be >= 0");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(ORBGPU_ERR_NO_DEVICE, "no HIP device visible");
    if (device >= n)
        return fail(ORBGPU_ERR_ARG, "device ordinal " + std::to_string(device) + " >= visible devices (" +
                                        std::to_string(n) + ")");
    return ORBGPU_OK;
}

}  // namespace orbgpu

namespace {

// OpenCV 2.4 cvRound / cvFloor on the host (SSE2 cvtsd2si = half to even)
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline int cv_floor(double v) { const int i = cv_round(v); return i - (v < (double)i); }
inline int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }


int vresize_simd_end(int width) {
    int x = 0;
    while (x <= width - 16) x += 16;
    while (x < width - 4) x += 4;
    return x;
}

// resize(src sw x sh -> dw x dh, INTER_LINEAR) tap tables, as cv::resize
// (2.4, imgwarp.cpp) computes xofs/ialpha and yofs/ibeta for 8U.
void build_resize_tables(int sw, int sh, int dw, int dh, std::vector<int2>& xt, std::vector<int2>& yt) {
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double scale_x = 1.0 / inv_sx, scale_y = 1.0 / inv_sy;
    xt.resize(dw);
    yt.resize(dh);
    int xmax = dw;
    std::vector<int> sxs(dw), a0s(dw), a1s(dw);
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= (float)sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
        }
        sxs[dx] = sx;
        a0s[dx] = sat_s16(cv_round((1.f - fx) * 2048.f));
        a1s[dx] = sat_s16(cv_round(fx * 2048.f));
    }
    for (int dx = 0; dx < dw; ++dx) {
        int sx0 = sxs[dx], sx1 = sxs[dx] + 1, a0 = a0s[dx], a1 = a1s[dx];
        if (dx >= xmax) { sx1 = sx0; a0 = 2048; a1 = 0; }  // HResizeLinear tail: S[sx]*ONE
        xt[dx].x = sx0 | (sx1 << 16);
        xt[dx].y = (a0 & 0xFFFF) | (a1 << 16);
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= (float)sy;
        const int b0 = sat_s16(cv_round((1.f - fy) * 2048.f)), b1 = sat_s16(cv_round(fy * 2048.f));
        const int y0 = std::min(std::max(sy, 0), sh - 1), y1 = std::min(std::max(sy + 1, 0), sh - 1);
        yt[dy].x = y0 | (y1 << 16);
        yt[dy].y = (b0 & 0xFFFF) | (b1 << 16);
    }
}

template <class T>
int dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    ORB_HIP(hipMalloc((void**)p, count * sizeof(T)));
    return ORBGPU_OK;
}

}  // namespace

struct orbgpu_extractor {
    Geom g;
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    float scale_factor = 0.f;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    int W = 0, H = 0, max_batch = 0, max_kps = 0;
    int ncap = 0;
    OctreeGroup oct_groups[2] = {};  // the octree launches (big levels / small levels)
    // device buffers
    uint8_t* d_pyr = nullptr;
    size_t pyr_bytes = 0;
    uint8_t* d_blur = nullptr;
    size_t blur_bytes = 0;
    int4* d_ptab = nullptr;
    PyrPlan pyr_plan;              // fused pyramid pass: row records, tick ranges, per-lane entries
    int4* d_pyr_ent = nullptr;
    int2* d_pyr_tab = nullptr;
    int2* d_xtab = nullptr;  // level-by-level pyramid (small batches): column / row taps per level
    int2* d_ytab = nullptr;
    int4* d_band = nullptr;  // banded pyramid (small batches): per band and level row ranges
    uint32_t* d_cand = nullptr;
    int* d_cell_counts = nullptr;
    uint32_t* d_gkeys = nullptr;
    uint16_t* d_gknode = nullptr;
    uint32_t* d_oct_out = nullptr;
    uint32_t* d_tab = nullptr;     // cell_tab then slot_tab (Geom)
    int* d_oct_count = nullptr;
    int* d_err = nullptr;
    int* d_trace = nullptr;  // optional octree pass trace (debug API)
    // ComputeStereoMatches: accepted SAD per left keypoint (pairs x cap), one scratch per
    // stream the batch form was called on (calls on different streams never share one)
    struct SadScratch {
        hipStream_t stream;
        int* d;
        size_t n;
    };
    std::vector<SadScratch> stereo_sad;
    std::mutex stereo_mu;
    // host-image path
    uint8_t* d_img = nullptr;
    uint8_t* fg_img = nullptr;  // host-mapped fine-grained HBM staging of the single-frame upload (knob)
    size_t img_pitch = 0;
    // one device block [count, err, pad, pad | keypoints(cap) | descriptors(cap)]
    // mirrored by one pinned host block, so a frame's outputs come back in a
    // single asynchronous copy
    uint8_t* d_single = nullptr;
    uint8_t* h_single = nullptr;  // pinned
    uint8_t* h_img = nullptr;     // pinned staging of the host image (img_pitch rows)
    unsigned long long* h_done = nullptr;  // pinned coherent: the single-frame completion flag (done_flag_kernel)
    unsigned long long done_seq = 0;       // the last issued call's flag value (0: none pending)
    uint8_t* h_levels = nullptr;  // pinned staging of one frame's pyramid (copy_levels), on first use
    size_t single_bytes = 0, single_desc_off = 0;
    orbgpu_keypoint* d_kps1 = nullptr;
    uint8_t* d_desc1 = nullptr;
    int* d_count1 = nullptr;
    hipStream_t stream = nullptr;
    // octree / describe chunk pipeline (run_batch): describe of chunk c on aux_stream
    // while the octree of chunk c+1 runs on the batch stream
    hipStream_t aux_stream = nullptr;
    std::array<hipEvent_t, 9> od_ev{};  // [c]: octree of chunk c done; [8]: the describes done
    // stage timing
    bool profile = false;
    int device = -1;  // the HIP device the handle's buffers and stream live on
    hipEvent_t stage_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // orbgpu_extractor_set_stage_event
    std::vector<std::array<hipEvent_t, 5>> ev;
    size_t ev_used = 0;
    // last extraction (for copy_level)
    const uint8_t* last_img = nullptr;
    size_t last_row = 0, last_frame = 0;
    int last_batch = 0;

    ~orbgpu_extractor() {
        DeviceScope ds(device);
        void* ptrs[] = {d_pyr, d_blur, d_ptab, d_pyr_ent, d_pyr_tab, d_xtab, d_ytab, d_band, d_cand, d_cell_counts, d_gkeys, d_gknode, d_oct_out,
                        d_oct_count, d_err, d_trace, d_img, fg_img, d_single, d_tab};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        for (auto& sc : stereo_sad) (void)hipFree(sc.d);
        if (h_single) (void)hipHostFree(h_single);
        if (h_img) (void)hipHostFree(h_img);
        if (h_done) (void)hipHostFree(h_done);
        if (h_levels) (void)hipHostFree(h_levels);
        if (stream) (void)hipStreamDestroy(stream);
        if (aux_stream) (void)hipStreamDestroy(aux_stream);
        for (hipEvent_t x : od_ev)
            if (x) (void)hipEventDestroy(x);
        for (auto& a : ev)
            for (hipEvent_t x : a) (void)hipEventDestroy(x);
    }
};

namespace {

// row pitch of pyramid levels >= 1 in HBM (bytes)
#ifndef ORBGPU_PYR_PITCH_ALIGN
#define ORBGPU_PYR_PITCH_ALIGN 16
#endif

// ORBextractor ctor arithmetic (ORBextractor.cpp:417-448) + per-level layout.
int build_geometry(orbgpu_extractor* e, std::vector<int4>& ptab, std::vector<int2>& ytab, std::vector<int2>* xtab) {
    const int L = e->nlevels;
    e->scale.assign(L, 1.f);
    e->sigma2.assign(L, 1.f);
    for (int i = 1; i < L; ++i) {
        e->scale[i] = e->scale[i - 1] * e->scale_factor;
        e->sigma2[i] = e->scale[i] * e->scale[i];
    }
    e->inv_scale.resize(L);
    e->inv_sigma2.resize(L);
    for (int i = 0; i < L; ++i) {
        e->inv_scale[i] = 1.0f / e->scale[i];
        e->inv_sigma2[i] = 1.0f / e->sigma2[i];
    }
    std::vector<int> nfeat(L);
    const float factor = 1.0f / e->scale_factor;
    float per_scale = e->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; ++l) {
        nfeat[l] = cv_round(per_scale);
        sum += nfeat[l];
        per_scale *= factor;
    }
    nfeat[L - 1] = std::max(e->nfeatures - sum, 0);

    Geom& g = e->g;
    std::memset(&g, 0, sizeof(g));
    g.nlevels = L;
    g.width = e->W;
    g.height = e->H;
    g.ini_th = std::min(std::max(e->ini_th, 0), 255);
    g.min_th = std::min(std::max(e->min_th, 0), 255);
    size_t pyr_off = 0, cand_off = 0;
    int cell_base = 0, out_off = 0, max_cells = 0, ncap = 0;
    ptab.clear();
    ytab.clear();
    if (xtab) xtab->clear();
    for (int l = 0; l < L; ++l) {
        LevelGeom& v = g.lv[l];
        v.w = cv_round((float)e->W * e->inv_scale[l]);
        v.h = cv_round((float)e->H * e->inv_scale[l]);
        v.scale = e->scale[l];
        v.size_i = (int)(31 * e->scale[l]);
        v.nfeat = nfeat[l];
        v.pitch = (int)round_up((size_t)v.w, l == 0 ? 16 : ORBGPU_PYR_PITCH_ALIGN);
        if (l > 0) {
            v.frame_bytes = (size_t)v.pitch * v.h;
            v.offset = pyr_off;
            pyr_off += round_up(v.frame_bytes * e->max_batch, 256);
        }
        // cells
        v.max_bx = v.w - kEdge + 3;
        v.max_by = v.h - kEdge + 3;
        const float width = (float)(v.max_bx - kBorder), height = (float)(v.max_by - kBorder);
        if (!(width >= 30.f && height >= 30.f))
            return fail(ORBGPU_ERR_UNSUPPORTED, "level " + std::to_string(l) + " is smaller than one FAST cell");
        v.ncols = (int)(width / 30.f);
        v.nrows = (int)(height / 30.f);
        v.wcell = (int)std::ceil(width / v.ncols);
        v.hcell = (int)std::ceil(height / v.nrows);
        if (v.wcell + 9 > kMaxWin || v.hcell + 6 > kMaxWin)
            return fail(ORBGPU_ERR_UNSUPPORTED, "FAST cell window larger than the LDS tile");
        if (v.max_bx - kBorder > 2047 || v.max_by - kBorder > 2047)
            return fail(ORBGPU_ERR_UNSUPPORTED, "levels wider/taller than 2079 px are not supported");
        v.cell_base = cell_base;
        v.cell_cap = ((v.wcell + 1) / 2) * ((v.hcell + 1) / 2);
        v.cand_offset = cand_off;
        cell_base += v.ncols * v.nrows;
        cand_off += (size_t)v.ncols * v.nrows * v.cell_cap;
        max_cells = std::max(max_cells, v.ncols * v.nrows);
        // octree roots (:545-547)
        v.nini = (int)std::round((float)(v.max_bx - kBorder) / (float)(v.max_by - kBorder));
        if (v.nini < 1) return fail(ORBGPU_ERR_UNSUPPORTED, "image aspect gives zero initial octree nodes");
        v.hx = (float)(v.max_bx - kBorder) / v.nini;
        v.ocap = std::max(v.nfeat + 3, 4 * v.nini);
        v.out_offset = out_off;
        out_off += v.ocap;
        ncap = std::max(ncap, std::max(v.ocap, v.nini));
        // resize tables: ytab rows as built; columns as per-quad tap records
        // for pyramid.hip (3 int4 per quad: (lo, wt) x 4 and the 4 perm selectors)
        if (l > 0) {
            const LevelGeom& p = g.lv[l - 1];
            std::vector<int2> xt, yt;
            build_resize_tables(p.w, p.h, v.w, v.h, xt, yt);
            for (const int2& t : xt)  // Q11 weights: non-negative, a0 + a1 = 2048 (+-1)
                if ((t.y & 0xFFFF) > 2049 || (t.y >> 16) < 0 || (t.y & 0xFFFF) + (t.y >> 16) > 2049)
                    return fail(ORBGPU_ERR_UNSUPPORTED, "unexpected resize weights");
            v.simd_end = vresize_simd_end(v.w);
            const int quads = (v.w + 3) / 4;
            if (quads < 3) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid level narrower than 9 px");
            // pyramid.hip gives the last quad (the scalar tail) its own lanes
            // (or, when w is a multiple of 16, there is no tail at all)
            if (v.simd_end == v.w && v.w % 4 == 0) v.qmain = quads;
            else if (v.simd_end == 4 * (quads - 1)) v.qmain = quads - 1;
            else return fail(ORBGPU_ERR_UNSUPPORTED, "resize tail is not the last quad");
            if ((size_t)v.pitch * v.h >= (1u << 31)) return fail(ORBGPU_ERR_UNSUPPORTED, "level too large");
            v.ptab_offset = (int)ptab.size();
            // Column taps per quad for pyramid.hip (3 int4 per quad):
            //   (w0, wt0, wt1, wt2), (wt3, sel0, sel1, sel2), (sel3, 0, 0, 0).
            // The kernel reads the three dwords d0, d1, d2 at byte w0 of the
            // source row; pixels 0..2 take their two taps from (d1:d0) and
            // pixel 3 from (d2:d1) with v_perm_b32 (selector sel_k puts the
            // tap bytes in the HIGH byte of each 16-bit lane, i.e. x256), and
            // wt_k = (16 ialpha0, 16 ialpha1) so v_dot2_u32_u16 yields
            // 4096 x the exact HResizeLinear sum: its high half is h >> 4,
            // the operand of VResizeLinearVec_32s8u.  w0 may be -4 or -8
            // (the LDS ring rows have 16 bytes in front).  Holds for every
            // scale factor <= 2 (checked here per quad).
            for (int q = 0; q < quads; ++q) {
                const int lo = xt[4 * q].x & 0xFFFF;
                int w0 = 0, sel[4] = {0, 0, 0, 0};
                bool ok = false;
                for (int c = 0; c < 3 && !ok; ++c) {
                    w0 = (lo & ~3) - 4 * c;
                    ok = true;
                    for (int k = 0; k < 4; ++k) {
                        const int dx = 4 * q + k;
                        if (dx >= v.w) { sel[k] = (int)0x0c0c0c0cu; continue; }
                        const int base = w0 + (k == 3 ? 4 : 0);
                        const int t0 = (xt[dx].x & 0xFFFF) - base;
                        const int t1 = ((xt[dx].y >> 16) != 0 ? (xt[dx].x >> 16) : (xt[dx].x & 0xFFFF)) - base;
                        if (t0 < 0 || t1 > 7 || t1 < t0) { ok = false; break; }
                        sel[k] = (int)(0x000c000cu | ((uint32_t)t0 << 8) | ((uint32_t)t1 << 24));
                    }
                }
                if (!ok) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid column taps do not fit a 12-byte window (scale factor > 2?)");
                if (q > 0 && w0 < 0) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid column window before the row start");
                int wt[4];
                for (int k = 0; k < 4; ++k) {
                    const int dx = 4 * q + k;
                    const uint32_t a0 = dx < v.w ? (uint32_t)(xt[dx].y & 0xFFFF) : 0u;
                    const uint32_t a1 = dx < v.w ? (uint32_t)(xt[dx].y >> 16) : 0u;
                    wt[k] = (int)((a0 << 4) | (a1 << 20));
                }
                ptab.push_back(int4{w0, wt[0], wt[1], wt[2]});
                ptab.push_back(int4{wt[3], sel[0], sel[1], sel[2]});
                ptab.push_back(int4{sel[3], 0, 0, 0});
            }
            v.ytab_offset = (int)ytab.size();
            ytab.insert(ytab.end(), yt.begin(), yt.end());
            if (xtab) {
                v.xtab_offset = (int)xtab->size();
                xtab->insert(xtab->end(), xt.begin(), xt.end());
            }
        }
    }
    {
        const int rc = plan_pyramid(g, ytab, ptab, e->max_batch, e->pyr_plan);
        if (rc) return rc;
    }
    g.total_cells = cell_base;
    g.cand_frame = cand_off;
    g.slots_frame = out_off;
    g.cells_magic = udiv40_magic((uint32_t)cell_base);
    g.slots_magic = udiv40_magic((uint32_t)out_off);
    for (int l = 0; l < kMaxLevels; ++l) {
        g.lvl_cell_base[l] = l < L ? g.lv[l].cell_base : INT_MAX;
        g.lvl_out_offset[l] = l < L ? g.lv[l].out_offset : INT_MAX;
    }
    g.max_cells_level = max_cells;
    size_t blur_off = 0;
    int tiles = 0;
    for (int l = 0; l < L; ++l) {
        LevelGeom& v = g.lv[l];
        v.blur_frame_bytes = (size_t)v.pitch * v.h;
        v.blur_offset = blur_off;
        blur_off += round_up(v.blur_frame_bytes * e->max_batch, 256);
        v.blur_tiles_x = (v.w + 3) / 4;
        v.blur_tile_base = tiles;
        tiles += v.blur_tiles_x * ((v.h + kBlurStrip - 1) / kBlurStrip);
    }
    g.blur_tiles_frame = tiles;
    e->blur_bytes = blur_off + 256;  // slack: describe reads 40-byte row spans
    g.win_pitch = 0;
    g.win_rows = 0;
    g.det_max = 0;
    for (int l = 0; l < L; ++l) {
        if (g.lv[l].wcell > 61) return fail(ORBGPU_ERR_UNSUPPORTED, "FAST cell wider than 61 px");
        // window = cell + 6 px, starting at tile column 1 or 5 (fast.hip's column shift)
        g.win_pitch = std::max(g.win_pitch, (int)round_up((size_t)g.lv[l].wcell + 11, 4));
        g.win_rows = std::max(g.win_rows, g.lv[l].hcell + 6);
        g.det_max = std::max(g.det_max, (int)round_up((size_t)g.lv[l].wcell * g.lv[l].hcell, 8));
    }
    // fast.hip is instantiated for window pitches 40, 48, ..., 72 (compile-time
    // ring offsets)
    g.win_pitch = g.win_pitch <= 40 ? 40 : (int)round_up((size_t)g.win_pitch, 8);
    e->pyr_bytes = pyr_off;
    e->max_kps = out_off;
    e->ncap = (int)round_up((size_t)ncap, 16);
    if (e->ncap > 4096) return fail(ORBGPU_ERR_UNSUPPORTED, "more than 4092 features per level");
    // octree.hip's main pass scans (children << 16 | survives) in one int:
    // C <= 4 * nodes must stay below 2^15 and S <= nodes below 2^16
    static_assert(4 * 4096 < (1 << 15), "octree packed scan bound");
    if (4 * e->ncap >= (1 << 15)) return fail(ORBGPU_ERR_UNSUPPORTED, "octree node capacity exceeds the packed scan");
    // Key capacity (a multiple of 64) for a requested one: the keys and their node
    // indices (6 bytes a key) in the requested LDS bytes less 64, and the whole
    // workgroup within 64 KiB; a level with more candidates uses HBM scratch.
    // keys in LDS (4 B key + 2 B node id each) for a request of `req` keys, in
    // steps of 64, shrunk until the workgroup's LDS fits 64 KiB: a request of
    // 2560 yields 2560 (round 5 subtracted a leftover 64 B and got 2496)
    auto key_capacity = [&g](int req, int ncap_) {
        const long bytes = (long)round_up((size_t)req * 4, 16) + (long)round_up((size_t)req * 2, 16);
        int kc = bytes > 0 ? (int)(bytes / 6) & ~63 : 0;
        while (kc > 0 && octree_lds_bytes(g, kc, ncap_) > 65536) kc -= 64;
        return kc;
    };
    // Two level groups in one octree launch: levels 0..1 (below), the
    // smaller levels with node arrays for their own feature counts and keys in LDS up to
    // ~2048; a level with more candidates takes the same HBM-scratch path as an oversized
    // big level.  The launch's LDS per workgroup is the larger group's.
    const int split = std::min(2, L);
    int ncap_b = 0;
    for (int l = split; l < L; ++l) ncap_b = std::max(ncap_b, std::max(g.lv[l].ocap, g.lv[l].nini));
    ncap_b = (int)round_up((size_t)std::max(ncap_b, 1), 16);
    // levels 0..1: keys in LDS up to ~2560 (26.1 KiB at 640x480: six workgroups per CU;
    // with 4096, four -- round 5: octree 0.158 -> 0.136 ms per 512 frames,
    // profiles/r05_notes_ab.txt r6c, r7a).  The bench stream's levels 0-1 have
    // ~1,000-1,300 candidates; a level with more than the capacity takes the HBM-scratch
    // path (correct, slower), as an oversized level always did.  ORBGPU_OCT_KCAP_A
    // overrides the 2560 (256..4096).
    const int kcap_a_req = [] {
        const char* s = std::getenv("ORBGPU_OCT_KCAP_A");
        const int v = s ? std::atoi(s) : 2560;
        return v >= 256 && v <= 4096 ? v : 2560;
    }();
    e->oct_groups[0] = OctreeGroup{0, split, key_capacity(kcap_a_req, e->ncap), e->ncap};
    e->oct_groups[1] = OctreeGroup{split, L - split, key_capacity(2048, ncap_b), ncap_b};
    return ORBGPU_OK;
}

// batches up to this size take the level-by-level pyramid (ORBGPU_PYR_LEVELS_MAX_BATCH overrides)
int pyr_levels_max_batch() {
    static const int v = [] {
        const char* s = std::getenv("ORBGPU_PYR_LEVELS_MAX_BATCH");
        return s ? std::atoi(s) : 8;
    }();
    return v;
}

// chunks of the octree / describe pipeline (ORBGPU_OD_CHUNKS, 1..8; 1 = the plain
// sequence): the octree of chunk c+1 (latency bound) runs beside the describe of
// chunk c (VALU bound)
int od_chunks() {  // read per batch (a test switches it within one process)
    const char* s = std::getenv("ORBGPU_OD_CHUNKS");
    const int n = s ? std::atoi(s) : 1;
    return n < 1 ? 1 : (n > 8 ? 8 : n);
}

// the single-frame path moves the frame in and the results out by kernels over
// PCIe (a copy kernel reading pinned memory; describe writing the results into
// pinned memory) -- ORBGPU_SINGLE_ZEROCOPY=0 selects copy-engine transfers
bool single_zero_copy() {
    static const bool v = [] {
        const char* s = std::getenv("ORBGPU_SINGLE_ZEROCOPY");
        return !(s && std::atoi(s) == 0);
    }();
    return v;
}

// the single-frame call waits on a completion flag written by a one-wave kernel
// after the extraction (ORBGPU_SINGLE_DONE_FLAG=0: hipStreamSynchronize)
bool single_done_flag() {
    static const bool v = [] {
        const char* s = std::getenv("ORBGPU_SINGLE_DONE_FLAG");
        return !(s && std::atoi(s) == 0);
    }();
    return v;
}

// The single-frame upload: the host writes the frame straight into host-mapped
// fine-grained HBM (write-combined over PCIe, ~7.5 us for 640x480) and the
// extraction reads it there -- no copy kernel (a memcpy into pinned memory,
// 2 us, then a copy kernel reading it over PCIe, 9.5 us).  Drop-in
// ORBextractor::operator() 87-91 -> 78-81 us with the completion flag
// (profiles/r06_notes_ab.txt r6p).  ORBGPU_SINGLE_VRAM_STAGING=0, or an
// allocation the device refuses: the pinned staging and the copy kernel.
bool single_vram_staging() {
    static const bool v = [] {
        const char* s = std::getenv("ORBGPU_SINGLE_VRAM_STAGING");
        return !(s && std::atoi(s) == 0);
    }();
    return v;
}

// ORBGPU_PYR_BANDS=0 selects the level-by-level launches (A/B and parity checks)
bool pyr_bands_off() {
    static const bool v = [] {
        const char* s = std::getenv("ORBGPU_PYR_BANDS");
        return s && std::atoi(s) == 0;
    }();
    return v;
}

int run_batch(orbgpu_extractor* e, const uint8_t* imgs, int batch, size_t row_step, size_t frame_step,
              orbgpu_keypoint* kps, uint8_t* desc, int* counts, int kp_cap, hipStream_t s, int* err_copy = nullptr) {
    const Geom& g = e->g;
    hipEvent_t* evs = nullptr;
    if (e->profile) {
        if (e->ev_used == e->ev.size()) {
            std::array<hipEvent_t, 5> a;
            // (timing only: no system-scope fence on record, which stalled the
            // stream before its next kernel)
            for (hipEvent_t& x : a) ORB_HIP(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
            e->ev.push_back(a);
        }
        evs = e->ev[e->ev_used++].data();
        ORB_HIP(hipEventRecord(evs[0], s));
    }
    // the tick pipeline is one block per frame: a few frames go in row bands
    // over the chip (one launch), or level by level when no band plan fits
    if (batch <= pyr_levels_max_batch() && g.bd_nb > 0 && !pyr_bands_off())
        ORB_HIP(launch_pyramid_bands(g, batch, e->d_band, e->d_xtab, e->d_ytab, imgs, row_step, frame_step, e->d_pyr, s));
    else if (batch <= pyr_levels_max_batch())
        ORB_HIP(launch_pyramid_levels(g, batch, e->d_xtab, e->d_ytab, imgs, row_step, frame_step, e->d_pyr, s));
    else
        ORB_HIP(launch_pyramid(g, batch, e->d_pyr_ent, e->d_pyr_tab, imgs, row_step, frame_step, e->d_pyr, s));
    if (evs) ORB_HIP(hipEventRecord(evs[1], s));
    if (e->stage_ev[0]) ORB_HIP(hipEventRecord(e->stage_ev[0], s));
    ORB_HIP(launch_fast_cells(g, batch, imgs, row_step, frame_step, e->d_pyr, e->d_cand, e->d_cell_counts, e->d_err, s));
    if (evs) ORB_HIP(hipEventRecord(evs[2], s));
    if (e->stage_ev[1]) ORB_HIP(hipEventRecord(e->stage_ev[1], s));
    const int nch = (err_copy || batch < 16 * od_chunks()) ? 1 : od_chunks();
    if (nch == 1) {
        ORB_HIP(launch_octree(g, batch, e->d_cand, e->d_cell_counts, e->d_gkeys, e->d_gknode, e->d_oct_out,
                              e->d_oct_count, e->d_err, e->oct_groups, 2, e->d_trace, s));
        if (evs) ORB_HIP(hipEventRecord(evs[3], s));
        if (e->stage_ev[2]) ORB_HIP(hipEventRecord(e->stage_ev[2], s));
        // GaussianBlur is fused into describe (blur of each keypoint's patch);
        // whole blurred levels exist only for the debug API (round 5: blurring
        // the upper levels whole and sampling them was slower)
        ORB_HIP(launch_describe(g, batch, imgs, row_step, frame_step, e->d_pyr, e->d_oct_out, e->d_oct_count, kps,
                                desc, counts, kp_cap, s, err_copy ? e->d_err : nullptr, err_copy));
    } else {
        // the octree chunks in order on s, each chunk's describe on the aux stream after
        // its octree: describe(c) overlaps octree(c+1); s joins the aux stream at the end
        if (!e->aux_stream) {
            int lo = 0, hi = 0;
            ORB_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
            ORB_HIP(hipStreamCreateWithPriority(&e->aux_stream, hipStreamNonBlocking, hi));
            for (hipEvent_t& x : e->od_ev) ORB_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        }
        hipStream_t a = e->aux_stream;
        for (int c = 0; c < nch; ++c) {
            const int f0 = batch * c / nch, f1 = batch * (c + 1) / nch, nb = f1 - f0;
            ORB_HIP(launch_octree(g, nb, e->d_cand + (size_t)f0 * g.cand_frame,
                                  e->d_cell_counts + (size_t)f0 * g.total_cells,
                                  e->d_gkeys + (size_t)f0 * g.cand_frame, e->d_gknode + (size_t)f0 * g.cand_frame,
                                  e->d_oct_out + (size_t)f0 * g.slots_frame, e->d_oct_count + (size_t)f0 * kOcStride,
                                  e->d_err, e->oct_groups, 2, c == 0 ? e->d_trace : nullptr, s));
            // the octree stage ends with the last chunk's octree (the describes of the
            // earlier chunks overlap it on the aux stream; describe = the rest)
            if (c == nch - 1 && evs) ORB_HIP(hipEventRecord(evs[3], s));
            ORB_HIP(hipEventRecord(e->od_ev[c], s));
            ORB_HIP(hipStreamWaitEvent(a, e->od_ev[c], 0));
            ORB_HIP(launch_describe(g, nb, imgs, row_step, frame_step, e->d_pyr, e->d_oct_out, e->d_oct_count, kps,
                                    desc, counts, kp_cap, a, nullptr, nullptr, f0));
        }
        if (e->stage_ev[2]) ORB_HIP(hipEventRecord(e->stage_ev[2], s));
        ORB_HIP(hipEventRecord(e->od_ev[8], a));
        ORB_HIP(hipStreamWaitEvent(s, e->od_ev[8], 0));
    }
    if (evs) ORB_HIP(hipEventRecord(evs[4], s));
    if (e->stage_ev[3]) ORB_HIP(hipEventRecord(e->stage_ev[3], s));
    e->last_img = imgs;
    e->last_row = row_step;
    e->last_frame = frame_step;
    e->last_batch = batch;
    return ORBGPU_OK;
}

std::string capacity_message(int err) {
    std::string m = "kernel capacity overflow:";
    if (err & kErrCellCap) m += " FAST-cell";
    if (err & kErrNodeCap) m += " octree-nodes";
    if (err & kErrKeyCap) m += " octree-keys";
    if (err & kErrSeqCap) m += " octree-seq";
    return m;
}

int collect_errors(orbgpu_extractor* e, hipStream_t s) {
    ORB_HIP(hipStreamSynchronize(s));
    int err = 0;
    ORB_HIP(hipMemcpy(&err, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (err) {
        ORB_HIP(hipMemset(e->d_err, 0, sizeof(int)));
        return fail(ORBGPU_ERR_CAPACITY, capacity_message(err));
    }
    return ORBGPU_OK;
}

}  // namespace

extern "C" {

const char* orbgpu_last_error(void) { return g_err.c_str(); }

int orbgpu_device_arch(char* buf, int buflen) {
    int dev = 0, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(ORBGPU_ERR_NO_DEVICE, "no HIP device visible");
    ORB_HIP(hipGetDevice(&dev));
    hipDeviceProp_t p;
    ORB_HIP(hipGetDeviceProperties(&p, dev));
    if (buf && buflen > 0) {
        std::strncpy(buf, p.gcnArchName, (size_t)buflen - 1);
        buf[buflen - 1] = 0;
    }
    return ORBGPU_OK;
}

int orbgpu_extractor_create(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th, int width,
                            int height, int max_batch, orbgpu_extractor** out) {
    if (!out) return fail(ORBGPU_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (nfeatures <= 0 || nlevels <= 0 || nlevels > kMaxLevels || !(scale_factor > 1.f) || width <= 0 ||
        height <= 0 || max_batch <= 0)
        return fail(ORBGPU_ERR_ARG, "invalid extractor parameters");
    int rc = check_device();
    if (rc) return rc;
    orbgpu_extractor* e = new orbgpu_extractor();
    ORB_HIP(hipGetDevice(&e->device));
    e->nfeatures = nfeatures;
    e->scale_factor = scale_factor;
    e->nlevels = nlevels;
    e->ini_th = ini_th;
    e->min_th = min_th;
    e->W = width;
    e->H = height;
    e->max_batch = max_batch;
    std::vector<int4> ptab;
    std::vector<int2> ytab, xtab;
    rc = build_geometry(e, ptab, ytab, &xtab);
    if (rc) { delete e; return rc; }
    std::vector<int4> bands;
    plan_pyramid_bands(e->g, ytab, bands);
    const Geom& g = e->g;
    const size_t B = (size_t)max_batch;
    e->img_pitch = round_up((size_t)width, 16);
    if ((rc = dalloc(&e->d_pyr, e->pyr_bytes)) || (rc = dalloc(&e->d_ptab, ptab.size())) ||
        (rc = dalloc(&e->d_cand, g.cand_frame * B)) ||
        (rc = dalloc(&e->d_cell_counts, (size_t)g.total_cells * B)) || (rc = dalloc(&e->d_gkeys, g.cand_frame * B)) ||
        (rc = dalloc(&e->d_gknode, g.cand_frame * B)) || (rc = dalloc(&e->d_oct_out, (size_t)g.slots_frame * B)) ||
        (rc = dalloc(&e->d_oct_count, (size_t)kOcStride * B)) || (rc = dalloc(&e->d_err, 1)) ||
        (rc = dalloc(&e->d_img, e->img_pitch * height)) ||
        (rc = dalloc(&e->d_pyr_ent, e->pyr_plan.ent.size())) || (rc = dalloc(&e->d_pyr_tab, e->pyr_plan.tab.size())) ||
        (rc = dalloc(&e->d_xtab, xtab.size())) || (rc = dalloc(&e->d_ytab, ytab.size())) ||
        (rc = dalloc(&e->d_band, std::max<size_t>(bands.size(), 1))) ||
        (rc = dalloc(&e->d_tab, (size_t)g.total_cells + g.slots_frame))) {
        delete e;
        return rc;
    }
    {  // per-cell / per-slot lookup tables (Geom::cell_tab, slot_tab)
        std::vector<uint32_t> tab((size_t)g.total_cells + g.slots_frame);
        for (int l = 0; l < g.nlevels; ++l) {
            const LevelGeom& v = g.lv[l];
            for (int c = 0; c < v.ncols * v.nrows; ++c)
                tab[(size_t)v.cell_base + c] = (uint32_t)l | (uint32_t)(c / v.ncols) << 4 | (uint32_t)(c % v.ncols) << 18;
            for (int i = 0; i < v.ocap; ++i) tab[(size_t)g.total_cells + v.out_offset + i] = (uint32_t)l | (uint32_t)i << 4;
        }
        if (hipMemcpy(e->d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            delete e;
            return fail(ORBGPU_ERR_HIP, "table upload failed");
        }
        e->g.cell_tab = e->d_tab;
        e->g.slot_tab = e->d_tab + g.total_cells;
    }
    e->single_desc_off = round_up(16 + (size_t)e->max_kps * sizeof(orbgpu_keypoint), 256);
    e->single_bytes = e->single_desc_off + (size_t)e->max_kps * 32;
    if ((rc = dalloc(&e->d_single, e->single_bytes))) {
        delete e;
        return rc;
    }
    e->d_count1 = reinterpret_cast<int*>(e->d_single);
    e->d_kps1 = reinterpret_cast<orbgpu_keypoint*>(e->d_single + 16);
    e->d_desc1 = e->d_single + e->single_desc_off;
    // (the output block coherent with the flag: describe's stores go straight
    // to host memory, so the flag written after them orders them for the host)
    if (hipHostMalloc((void**)&e->h_single, e->single_bytes,
                      single_done_flag() ? hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&e->h_img, e->img_pitch * height, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&e->h_done, 64, hipHostMallocCoherent) != hipSuccess) {
        delete e;
        return fail(ORBGPU_ERR_HIP, "pinned staging allocation failed");
    }
    __atomic_store_n(e->h_done, 0ull, __ATOMIC_RELEASE);
    if (single_vram_staging() &&
        hipExtMallocWithFlags((void**)&e->fg_img, e->img_pitch * height, hipDeviceMallocFinegrained) != hipSuccess)
        e->fg_img = nullptr;  // (the pinned staging and the copy kernel then)
    if (hipMemcpy(e->d_ptab, ptab.data(), ptab.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess ||
        (!xtab.empty() && hipMemcpy(e->d_xtab, xtab.data(), xtab.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) ||
        (!ytab.empty() && hipMemcpy(e->d_ytab, ytab.data(), ytab.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) ||
        (!bands.empty() && hipMemcpy(e->d_band, bands.data(), bands.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) ||
        (!e->pyr_plan.ent.empty() && hipMemcpy(e->d_pyr_ent, e->pyr_plan.ent.data(),
                                               e->pyr_plan.ent.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) ||
        (!e->pyr_plan.tab.empty() && hipMemcpy(e->d_pyr_tab, e->pyr_plan.tab.data(),
                                               e->pyr_plan.tab.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) ||
        pyramid_set_lds_limit(g) != hipSuccess ||
        hipMemset(e->d_err, 0, sizeof(int)) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return fail(ORBGPU_ERR_HIP, "buffer initialisation failed");
    }
    *out = e;
    return ORBGPU_OK;
}

int orbgpu_extractor_create_on_device(int device, int nfeatures, float scale_factor, int nlevels, int ini_th,
                                      int min_th, int width, int height, int max_batch, orbgpu_extractor** out) {
    if (out) *out = nullptr;
    int rc = validate_device(device);
    if (rc) return rc;
    DeviceScope ds(device);
    return orbgpu_extractor_create(nfeatures, scale_factor, nlevels, ini_th, min_th, width, height, max_batch, out);
}

int orbgpu_extractor_destroy(orbgpu_extractor* e) {
    delete e;
    return ORBGPU_OK;
}

int orbgpu_device_count(int* n) {
    if (!n) return fail(ORBGPU_ERR_ARG, "n is NULL");
    *n = 0;
    if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
    return ORBGPU_OK;
}

int orbgpu_set_thread_device(int device) {
    int rc = validate_device(device);
    if (rc) return rc;
    ORB_HIP(hipSetDevice(device));
    return check_device();
}

int orbgpu_get_thread_device(int* device) {
    if (!device) return fail(ORBGPU_ERR_ARG, "device is NULL");
    *device = -1;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(ORBGPU_ERR_NO_DEVICE, "no HIP device visible");
    ORB_HIP(hipGetDevice(device));
    return ORBGPU_OK;
}

int orbgpu_abi_version(void) { return ORBGPU_ABI_VERSION; }

int orbgpu_extractor_get_info_sized(const orbgpu_extractor* e, orbgpu_extractor_info* info, size_t info_size) {
    if (!e || !info) return fail(ORBGPU_ERR_ARG, "NULL argument");
    if (info_size == 0) return fail(ORBGPU_ERR_ARG, "info_size is 0");
    orbgpu_extractor_info full;
    const int rc = orbgpu_extractor_get_info(e, &full);
    if (rc) return rc;
    std::memcpy(info, &full, std::min(info_size, sizeof(full)));
    return ORBGPU_OK;
}

int orbgpu_extractor_get_info(const orbgpu_extractor* e, orbgpu_extractor_info* info) {
    if (!e || !info) return fail(ORBGPU_ERR_ARG, "NULL argument");
    std::memset(info, 0, sizeof(*info));
    info->nlevels = e->nlevels;
    info->width = e->W;
    info->height = e->H;
    info->max_batch = e->max_batch;
    info->max_keypoints = e->max_kps;
    info->device = e->device;
    for (int l = 0; l < e->nlevels && l < 32; ++l) {
        info->level_width[l] = e->g.lv[l].w;
        info->level_height[l] = e->g.lv[l].h;
        info->features_per_level[l] = e->g.lv[l].nfeat;
        info->level_capacity[l] = e->g.lv[l].ocap;
    }
    return ORBGPU_OK;
}

int orbgpu_extractor_get_scales(const orbgpu_extractor* e, float* s, float* is, float* s2, float* is2) {
    if (!e) return fail(ORBGPU_ERR_ARG, "NULL extractor");
    for (int l = 0; l < e->nlevels; ++l) {
        if (s) s[l] = e->scale[l];
        if (is) is[l] = e->inv_scale[l];
        if (s2) s2[l] = e->sigma2[l];
        if (is2) is2[l] = e->inv_sigma2[l];
    }
    return ORBGPU_OK;
}

int orbgpu_extract_batch_device(orbgpu_extractor* e, const uint8_t* imgs, int batch, size_t row_step,
                                size_t frame_step, orbgpu_keypoint* kps, uint8_t* desc, int* counts,
                                int kp_cap, void* stream) {
    if (!e || !imgs || !kps || !desc || !counts) return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (batch <= 0 || batch > e->max_batch) return fail(ORBGPU_ERR_ARG, "batch outside [1, max_batch]");
    if (kp_cap < e->max_kps) return fail(ORBGPU_ERR_CAPACITY, "kp_capacity < max_keypoints");
    if (row_step < (size_t)e->W || row_step % 16 || ((uintptr_t)imgs & 15) || (batch > 1 && frame_step % 16) ||
        (batch > 1 && frame_step < row_step * e->H))
        return fail(ORBGPU_ERR_ARG, "images must be 16-byte aligned with row_step and frame_step multiples of 16");
    return run_batch(e, imgs, batch, row_step, frame_step, kps, desc, counts, kp_cap, (hipStream_t)stream);
}

int orbgpu_extractor_sync(orbgpu_extractor* e, void* stream) {
    if (!e) return fail(ORBGPU_ERR_ARG, "NULL extractor");
    DeviceScope ds_(e->device);
    return collect_errors(e, (hipStream_t)stream);
}

// orbgpu_extract in two halves: issue (host image -> staging -> HBM,
// extraction, results towards the pinned output block; nothing waited for)
// and finish (one stream synchronisation, then the results out of the pinned
// block).  orbgpu_extract_pair issues two extractors' frames from one thread
// before finishing either.
static int extract_issue(orbgpu_extractor* e, const uint8_t* image, int width, int height, size_t step) {
    if (width != e->W || height != e->H) return fail(ORBGPU_ERR_ARG, "image size differs from the extractor geometry");
    if (step < (size_t)width) return fail(ORBGPU_ERR_ARG, "step < width");
    hipStream_t s = e->stream;
    if (single_zero_copy()) {
        // the drop-in (Frame constructor) path without copy-engine transfers:
        // host image -> pinned staging (one memcpy for a continuous image) ->
        // a copy kernel into HBM; extraction with describe writing keypoints,
        // descriptors, the count and the error word straight into the pinned
        // output block
        uint8_t* stage = e->fg_img ? e->fg_img : e->h_img;
        if (step == e->img_pitch)
            std::memcpy(stage, image, step * (size_t)height);
        else
            for (int y = 0; y < height; ++y)
                std::memcpy(stage + (size_t)y * e->img_pitch, image + (size_t)y * step, width);
        if (!e->fg_img) ORB_HIP(launch_copy16(e->d_img, e->h_img, e->img_pitch * (size_t)height, s));
        const int rc = run_batch(e, e->fg_img ? e->fg_img : e->d_img, 1, e->img_pitch, e->img_pitch * height,
                                 reinterpret_cast<orbgpu_keypoint*>(e->h_single + 16), e->h_single + e->single_desc_off,
                                 reinterpret_cast<int*>(e->h_single), e->max_kps, s,
                                 reinterpret_cast<int*>(e->h_single + 4));
        if (rc || !single_done_flag()) return rc;
        static std::atomic<unsigned long long> next_seq{1};  // distinct across extractors and calls
        const unsigned long long seq = next_seq.fetch_add(1, std::memory_order_relaxed);
        ORB_HIP(launch_done_flag(e->h_done, seq, s));
        e->done_seq = seq;
        return ORBGPU_OK;
    }
    // the drop-in path with copy-engine transfers: host image -> pinned
    // staging -> one async H2D; extraction; the error word folded into the
    // output block; one async D2H of the whole block (in four row bands: the
    // DMA of band i overlaps the host copy of band i+1)
    constexpr int kBands = 4;
    for (int b = 0; b < kBands; ++b) {
        const int y0 = height * b / kBands, y1 = height * (b + 1) / kBands;
        if (y1 <= y0) continue;
        if (step == e->img_pitch)  // a continuous cv::Mat of a 16-multiple width: one copy per band
            std::memcpy(e->h_img + (size_t)y0 * step, image + (size_t)y0 * step, step * (size_t)(y1 - y0));
        else
            for (int y = y0; y < y1; ++y)
                std::memcpy(e->h_img + (size_t)y * e->img_pitch, image + (size_t)y * step, width);
        ORB_HIP(hipMemcpyAsync(e->d_img + (size_t)y0 * e->img_pitch, e->h_img + (size_t)y0 * e->img_pitch,
                               e->img_pitch * (size_t)(y1 - y0), hipMemcpyHostToDevice, s));
    }
    // describe moves the error word into the output block and clears it
    int rc = run_batch(e, e->d_img, 1, e->img_pitch, e->img_pitch * height, e->d_kps1, e->d_desc1, e->d_count1,
                       e->max_kps, s, reinterpret_cast<int*>(e->d_single + 4));
    if (rc) return rc;
    ORB_HIP(hipMemcpyAsync(e->h_single, e->d_single, e->single_bytes, hipMemcpyDeviceToHost, s));
    return ORBGPU_OK;
}

// the call's completion: its flag (spun on; after 20 ms, or with no flag
// pending, the stream is synchronised, which also reports a failed kernel)
static int wait_single(orbgpu_extractor* e) {
    const unsigned long long seq = e->done_seq;
    e->done_seq = 0;
    if (seq) {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned it = 1;; ++it) {
            if (__atomic_load_n(e->h_done, __ATOMIC_ACQUIRE) == seq) return ORBGPU_OK;
            if ((it & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
            __builtin_ia32_pause();
        }
    }
    ORB_HIP(hipStreamSynchronize(e->stream));
    return ORBGPU_OK;
}

static int extract_finish(orbgpu_extractor* e, orbgpu_keypoint* keypoints, uint8_t* descriptors, int capacity,
                          int* n) {
    if (int rc = wait_single(e)) return rc;
    int count = 0, err = 0;
    std::memcpy(&count, e->h_single, sizeof(int));
    std::memcpy(&err, e->h_single + 4, sizeof(int));
    if (err) return fail(ORBGPU_ERR_CAPACITY, capacity_message(err));
    if (count > capacity) return fail(ORBGPU_ERR_CAPACITY, "keypoint capacity too small");
    if (count > 0) {
        if (keypoints) std::memcpy(keypoints, e->h_single + 16, (size_t)count * sizeof(orbgpu_keypoint));
        if (descriptors) std::memcpy(descriptors, e->h_single + e->single_desc_off, (size_t)count * 32);
    }
    *n = count;
    return ORBGPU_OK;
}

int orbgpu_extract(orbgpu_extractor* e, const uint8_t* image, int width, int height, size_t step,
                   orbgpu_keypoint* keypoints, uint8_t* descriptors, int capacity, int* n) {
    if (!e || !n) return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (!image || width <= 0 || height <= 0) {  // ORBextractor.cpp:1056
        *n = -1;
        return ORBGPU_OK;
    }
    int rc = extract_issue(e, image, width, height, step);
    if (rc) return rc;
    return extract_finish(e, keypoints, descriptors, capacity, n);
}

int orbgpu_extract_pair(orbgpu_extractor* e0, const uint8_t* image0, size_t step0, orbgpu_keypoint* keypoints0,
                        uint8_t* descriptors0, int capacity0, int* n0, orbgpu_extractor* e1, const uint8_t* image1,
                        size_t step1, orbgpu_keypoint* keypoints1, uint8_t* descriptors1, int capacity1, int* n1,
                        int width, int height) {
    if (!e0 || !e1 || !n0 || !n1) return fail(ORBGPU_ERR_ARG, "NULL argument");
    if (e0 == e1) return fail(ORBGPU_ERR_ARG, "the two frames need two extractors");
    const bool empty = !image0 || !image1 || width <= 0 || height <= 0;
    if (empty) {  // ORBextractor.cpp:1056, per image
        *n0 = *n1 = -1;
        int rc = ORBGPU_OK;
        if (image0 && width > 0 && height > 0)
            rc = orbgpu_extract(e0, image0, width, height, step0, keypoints0, descriptors0, capacity0, n0);
        if (!rc && image1 && width > 0 && height > 0)
            rc = orbgpu_extract(e1, image1, width, height, step1, keypoints1, descriptors1, capacity1, n1);
        return rc;
    }
    int rc;
    {
        DeviceScope ds_(e0->device);
        rc = extract_issue(e0, image0, width, height, step0);
    }
    if (rc) {
        DeviceScope ds_(e0->device);
        (void)hipStreamSynchronize(e0->stream);  // nothing of frame 0 is left in flight
        return rc;
    }
    int rc1;
    {
        DeviceScope ds_(e1->device);
        rc1 = extract_issue(e1, image1, width, height, step1);
    }
    {
        DeviceScope ds_(e0->device);
        rc = extract_finish(e0, keypoints0, descriptors0, capacity0, n0);
    }
    DeviceScope ds_(e1->device);
    if (rc1) {
        (void)hipStreamSynchronize(e1->stream);
        return rc1;
    }
    const int r1 = extract_finish(e1, keypoints1, descriptors1, capacity1, n1);
    return rc ? rc : r1;
}

int orbgpu_extractor_profile(orbgpu_extractor* e, int enable) {
    if (!e) return fail(ORBGPU_ERR_ARG, "NULL extractor");
    e->profile = enable != 0;
    return ORBGPU_OK;
}

int orbgpu_extractor_set_stage_event(orbgpu_extractor* e, int stage, void* event) {
    if (!e || stage < 0 || stage > 3) return fail(ORBGPU_ERR_ARG, "invalid argument");
    e->stage_ev[stage] = (hipEvent_t)event;
    return ORBGPU_OK;
}

int orbgpu_device_event_create(void** event) {
    if (!event) return fail(ORBGPU_ERR_ARG, "NULL event");
    hipEvent_t e = nullptr;
    ORB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    *event = e;
    return ORBGPU_OK;
}

int orbgpu_device_event_destroy(void* event) {
    if (event) ORB_HIP(hipEventDestroy((hipEvent_t)event));
    return ORBGPU_OK;
}

int orbgpu_device_event_record(void* event, void* stream) {
    if (!event) return fail(ORBGPU_ERR_ARG, "NULL event");
    ORB_HIP(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_stream_wait_device_event(void* stream, void* event) {
    if (!event) return fail(ORBGPU_ERR_ARG, "NULL event");
    ORB_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
    return ORBGPU_OK;
}

int orbgpu_extractor_stage_times(orbgpu_extractor* e, float* ms4, int* nbatches, int reset) {
    if (!e) return fail(ORBGPU_ERR_ARG, "NULL extractor");
    DeviceScope ds_(e->device);
    float acc[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < e->ev_used; ++i) {
        ORB_HIP(hipEventSynchronize(e->ev[i][4]));
        for (int k = 0; k < 4; ++k) {
            float ms = 0.f;
            ORB_HIP(hipEventElapsedTime(&ms, e->ev[i][k], e->ev[i][k + 1]));
            acc[k] += ms;
        }
    }
    if (ms4)
        for (int k = 0; k < 4; ++k) ms4[k] = acc[k];
    if (nbatches) *nbatches = (int)e->ev_used;
    if (reset) e->ev_used = 0;
    return ORBGPU_OK;
}

int orbgpu_extractor_copy_level(orbgpu_extractor* e, int frame, int level, uint8_t* dst, size_t dst_step) {
    if (!e || !dst) return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (!e->last_img || frame < 0 || frame >= e->last_batch || level < 0 || level >= e->nlevels)
        return fail(ORBGPU_ERR_ARG, "no such frame/level in the last extraction");
    const LevelGeom& v = e->g.lv[level];
    if (dst_step < (size_t)v.w) return fail(ORBGPU_ERR_ARG, "dst_step < level width");
    const uint8_t* src = level == 0 ? e->last_img + (size_t)frame * e->last_frame
                                    : e->d_pyr + v.offset + (size_t)frame * v.frame_bytes;
    const size_t pitch = level == 0 ? e->last_row : (size_t)v.pitch;
    ORB_HIP(hipStreamSynchronize(e->stream));
    ORB_HIP(hipMemcpy2D(dst, dst_step, src, pitch, v.w, v.h, hipMemcpyDeviceToHost));
    return ORBGPU_OK;
}

// mvImagePyramid of one frame: every level into pinned staging with one async
// copy each on the extractor's stream, one synchronisation, then host copies
// into the caller's rows (a pageable 2-D copy per level costs ~1 ms)
int orbgpu_extractor_copy_levels(orbgpu_extractor* e, int frame, uint8_t* const* dst, const size_t* dst_step) {
    if (!e || !dst || !dst_step) return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (!e->last_img || frame < 0 || frame >= e->last_batch)
        return fail(ORBGPU_ERR_ARG, "no such frame in the last extraction");
    size_t total = 0, off[kMaxLevels];
    for (int l = 0; l < e->nlevels; ++l) {
        const LevelGeom& v = e->g.lv[l];
        if (!dst[l] || dst_step[l] < (size_t)v.w) return fail(ORBGPU_ERR_ARG, "bad destination of a level");
        off[l] = total;
        total += round_up((size_t)v.pitch * v.h, 256);
    }
    if (!e->h_levels) ORB_HIP(hipHostMalloc((void**)&e->h_levels, total, hipHostMallocDefault));
    // level 0 of the last single-frame call is still in the pinned upload
    // staging (pinned-staging path); other levels, and level 0 otherwise (the
    // fine-grained HBM staging, a batch), come back by one copy kernel writing
    // the pinned staging (no copy-engine transfers; a level 0 whose rows do not
    // fit the staging's level-0 pitch by a 2-D copy)
    const bool l0_host = single_zero_copy() && e->last_img == e->d_img && e->last_batch == 1;
    const uint8_t* l0_dev = e->last_img + (size_t)frame * e->last_frame;
    const bool l0_kernel = !l0_host && e->last_row <= (size_t)e->g.lv[0].pitch &&
                           (((uintptr_t)l0_dev | e->last_row * e->g.lv[0].h) & 15) == 0;
    if (!l0_host && !l0_kernel)
        ORB_HIP(hipMemcpy2DAsync(e->h_levels, (size_t)e->g.lv[0].pitch, l0_dev, e->last_row, e->g.lv[0].w,
                                 e->g.lv[0].h, hipMemcpyDeviceToHost, e->stream));
    if (e->nlevels > 1 || l0_kernel) {
        CopyList16 L{};
        L.n = 0;
        if (l0_kernel) L.d[L.n++] = CopyDesc16{l0_dev, e->h_levels + off[0], e->last_row * e->g.lv[0].h};
        for (int l = 1; l < e->nlevels && L.n < kCopyList; ++l) {
            const LevelGeom& v = e->g.lv[l];
            L.d[L.n++] = CopyDesc16{e->d_pyr + v.offset + (size_t)frame * v.frame_bytes, e->h_levels + off[l],
                                    (size_t)v.pitch * v.h};
        }
        ORB_HIP(launch_copy16_list(L, e->stream));
    }
    ORB_HIP(hipStreamSynchronize(e->stream));
    for (int l = 0; l < e->nlevels; ++l) {
        const LevelGeom& v = e->g.lv[l];
        const uint8_t* src = l == 0 && l0_host ? e->h_img : e->h_levels + off[l];
        const size_t sp = l == 0 && (l0_host || l0_kernel) ? (l0_host ? e->img_pitch : e->last_row) : (size_t)v.pitch;
        for (int y = 0; y < v.h; ++y) std::memcpy(dst[l] + (size_t)y * dst_step[l], src + (size_t)y * sp, (size_t)v.w);
    }
    return ORBGPU_OK;
}

int orbgpu_debug_level_blur(orbgpu_extractor* e, int frame, int level, uint8_t* dst, size_t dst_step) {
    if (!e || !dst) return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (!e->last_img || frame < 0 || frame >= e->last_batch || level < 0 || level >= e->nlevels)
        return fail(ORBGPU_ERR_ARG, "no such frame/level in the last extraction");
    const LevelGeom& v = e->g.lv[level];
    if (dst_step < (size_t)v.w) return fail(ORBGPU_ERR_ARG, "dst_step < level width");
    ORB_HIP(hipStreamSynchronize(e->stream));
    // the product path never materialises blurred levels: blur the last
    // batch's levels on demand (same arithmetic as describe's fused blur)
    if (!e->d_blur) {
        int rc = dalloc(&e->d_blur, e->blur_bytes);
        if (rc) return rc;
    }
    ORB_HIP(launch_blur_levels(e->g, e->last_batch, e->last_img, e->last_row, e->last_frame, e->d_pyr, e->d_blur,
                               e->stream));
    ORB_HIP(hipStreamSynchronize(e->stream));
    ORB_HIP(hipMemcpy2D(dst, dst_step, e->d_blur + v.blur_offset + (size_t)frame * v.blur_frame_bytes, v.pitch, v.w,
                        v.h, hipMemcpyDeviceToHost));
    return ORBGPU_OK;
}

int orbgpu_hamming_pairs_device(const uint8_t* a, const uint8_t* b, int n, int* dist, void* stream) {
    if (n < 0 || (n > 0 && (!a || !b || !dist))) return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (((uintptr_t)a | (uintptr_t)b) & 31) return fail(ORBGPU_ERR_ARG, "descriptors must be 32-byte aligned");
    ORB_HIP(launch_hamming_pairs(a, b, n, dist, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_pack_rows_device(int batch, int cap, int ntensors, const orbgpu_pack_desc* d, void* stream) {
    if (batch < 0 || cap < 0 || ntensors < 0 || ntensors > 4 || (ntensors > 0 && !d))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    for (int t = 0; t < ntensors; ++t)
        if (!d[t].rows || !d[t].packed || !d[t].counts || d[t].row_bytes <= 0 || (d[t].row_bytes & 3) ||
            (((uintptr_t)d[t].rows | (uintptr_t)d[t].packed) & 3))
            return fail(ORBGPU_ERR_ARG, "pack: rows must be 4-byte multiples at 4-byte aligned addresses");
    ORB_HIP(launch_pack_rows(batch, cap, ntensors, d, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_search_for_initialization_batch_device_bounded(
    int batch, orbgpu_grid_bounds bd, const orbgpu_keypoint* kps1, const uint8_t* desc1, const int* n1, size_t stride1,
    const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2, size_t stride2, float* prev_xy, int window,
    float nnratio, int flags, int max_level0, int* matches12, int* nmatches, void* stream) {
    if (batch <= 0 || !kps1 || !kps2 || !desc1 || !desc2 || !n1 || !n2 || !matches12 || !nmatches ||
        !(bd.max_x > bd.min_x) || !(bd.max_y > bd.min_y) || max_level0 < 0)
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    ORB_HIP(launch_match_init(batch, bd.min_x, bd.max_x, bd.min_y, bd.max_y, kps1, desc1, n1, stride1, kps2, desc2, n2, stride2, prev_xy,
                              window, nnratio, flags, matches12, nmatches, (hipStream_t)stream, (size_t)max_level0));
    return ORBGPU_OK;
}

int orbgpu_search_for_initialization_stream_device(int batch, orbgpu_grid_bounds bd, const orbgpu_keypoint* kps,
                                                   const uint8_t* desc, const int* n, size_t stride,
                                                   const orbgpu_keypoint* prev_kps, const uint8_t* prev_desc,
                                                   const int* prev_n, float* prev_xy, int window, float nnratio,
                                                   int flags, int max_level0, int* matches12, int* nmatches,
                                                   void* stream) {
    if (batch <= 0 || !kps || !desc || !n || !prev_kps || !prev_desc || !prev_n || !matches12 || !nmatches ||
        stride == 0 || !(bd.max_x > bd.min_x) || !(bd.max_y > bd.min_y) || max_level0 < 0)
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    MatchFirstF1 first;
    first.kps = prev_kps;
    first.desc = prev_desc;
    first.n = prev_n;
    ORB_HIP(launch_match_init(batch, bd.min_x, bd.max_x, bd.min_y, bd.max_y, kps, desc, n, stride, kps, desc, n,
                              stride, prev_xy, window, nnratio, flags, matches12, nmatches, (hipStream_t)stream,
                              (size_t)max_level0, first));
    return ORBGPU_OK;
}

int orbgpu_search_for_initialization_batch_device(int batch, orbgpu_grid_bounds bd, const orbgpu_keypoint* kps1,
                                                  const uint8_t* desc1, const int* n1, size_t stride1,
                                                  const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2,
                                                  size_t stride2, float* prev_xy, int window, float nnratio,
                                                  int flags, int* matches12, int* nmatches, void* stream) {
    return orbgpu_search_for_initialization_batch_device_bounded(batch, bd, kps1, desc1, n1, stride1, kps2, desc2, n2,
                                                                 stride2, prev_xy, window, nnratio, flags, 0,
                                                                 matches12, nmatches, stream);
}

int orbgpu_search_for_initialization(orbgpu_grid_bounds bd, const orbgpu_keypoint* kps1, const uint8_t* desc1,
                                     int n1, const orbgpu_keypoint* kps2, const uint8_t* desc2, int n2,
                                     float* prev_xy, int window, float nnratio, int flags, int* matches12,
                                     int* nmatches) {
    if (n1 < 0 || n2 < 0 || !matches12 || !nmatches) return fail(ORBGPU_ERR_ARG, "invalid argument");
    int rc = check_device();
    if (rc) return rc;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    const size_t n1c = std::max(n1, 1), n2c = std::max(n2, 1);
    const int ns[3] = {n1, n2, 0};
    const orbgpu_keypoint *dk1, *dk2;
    const uint8_t *dd1, *dd2;
    int *dn, *dm;
    float* dp;
    HostCall call(*ctx);
    rc = call.run([&](HostCall& A) {
        dk1 = A.inout(kps1, (size_t)n1, n1c);
        dk2 = A.inout(kps2, (size_t)n2, n2c);
        dd1 = A.inout(desc1, 32 * (size_t)n1, 32 * n1c);
        dd2 = A.inout(desc2, 32 * (size_t)n2, 32 * n2c);
        dn = A.inout(ns, 3);
        dm = A.out<int>(n1c);
        dp = prev_xy ? A.inout(prev_xy, 2 * (size_t)n1, 2 * n1c) : nullptr;
    });
    if (rc) return rc;
    // the number of level-0 keypoints bounds which matcher variants can be
    // needed, so a 1000-feature frame (~220 at level 0) takes one launch, not
    // one per variant (all octave-0 entries are counted: an upper bound of the
    // leading run the kernel uses, whatever the order)
    auto level0 = [](const orbgpu_keypoint* k, int n) {
        int c = 0;
        for (int i = 0; i < n; ++i) c += k[i].octave == 0;
        return c;
    };
    const size_t n0 = (size_t)std::max(std::max(level0(kps1, n1), level0(kps2, n2)), 1);
    if (!(bd.max_x > bd.min_x) || !(bd.max_y > bd.min_y)) return fail(ORBGPU_ERR_ARG, "invalid argument");
    ORB_HIP(launch_match_init(1, bd.min_x, bd.max_x, bd.min_y, bd.max_y, dk1, dd1, dn, n1c, dk2, dd2, dn + 1, n2c, dp,
                              window, nnratio, flags, dm, dn + 2, ctx->stream, n0));
    call.fetch(dm, matches12, (size_t)n1 * sizeof(int));
    call.fetch(dn + 2, nmatches, sizeof(int));
    if (prev_xy) call.fetch(dp, prev_xy, (size_t)n1 * 2 * sizeof(float));
    if ((rc = call.finish())) return rc;
    if (*nmatches < 0) {
        *nmatches = 0;
        return fail(ORBGPU_ERR_CAPACITY, "matcher: more than 2048 level-0 keypoints in a frame");
    }
    return ORBGPU_OK;
}

int orbgpu_debug_level_candidates(orbgpu_extractor* e, int frame, int level, int* xys, int cap) {
    if (!e || frame < 0 || frame >= e->last_batch || level < 0 || level >= e->nlevels)
        return fail(ORBGPU_ERR_ARG, "no such frame/level in the last extraction");
    DeviceScope ds_(e->device);
    const Geom& g = e->g;
    const LevelGeom& v = g.lv[level];
    const int ncells = v.ncols * v.nrows;
    std::vector<int> counts(ncells);
    std::vector<uint32_t> slots((size_t)ncells * v.cell_cap);
    ORB_HIP(hipStreamSynchronize(e->stream));
    ORB_HIP(hipDeviceSynchronize());
    ORB_HIP(hipMemcpy(counts.data(), e->d_cell_counts + (size_t)frame * g.total_cells + v.cell_base,
                      ncells * sizeof(int), hipMemcpyDeviceToHost));
    ORB_HIP(hipMemcpy(slots.data(), e->d_cand + (size_t)frame * g.cand_frame + v.cand_offset,
                      slots.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    int n = 0;
    for (int c = 0; c < ncells; ++c)
        for (int k = 0; k < counts[c]; ++k, ++n)
            if (n < cap && xys) {
                const uint32_t key = slots[(size_t)c * v.cell_cap + k];
                xys[3 * n] = key_x(key); xys[3 * n + 1] = key_y(key); xys[3 * n + 2] = key_s(key);
            }
    return n;
}

int orbgpu_debug_octree_trace(orbgpu_extractor* e, int enable, int* out, int cap) {
    if (!e) return fail(ORBGPU_ERR_ARG, "NULL extractor");
    DeviceScope ds_(e->device);
    const size_t n = (size_t)kMaxLevels * 512;
    if (enable && !e->d_trace) {
        ORB_HIP(hipMalloc((void**)&e->d_trace, n * sizeof(int)));
        ORB_HIP(hipMemset(e->d_trace, 0, n * sizeof(int)));
    }
    if (out && e->d_trace) {
        ORB_HIP(hipDeviceSynchronize());
        ORB_HIP(hipMemcpy(out, e->d_trace, std::min(n, (size_t)cap) * sizeof(int), hipMemcpyDeviceToHost));
    }
    return ORBGPU_OK;
}

int orbgpu_debug_level_octree(orbgpu_extractor* e, int frame, int level, int* xys, int cap) {
    if (!e || frame < 0 || frame >= e->last_batch || level < 0 || level >= e->nlevels)
        return fail(ORBGPU_ERR_ARG, "no such frame/level in the last extraction");
    DeviceScope ds_(e->device);
    const Geom& g = e->g;
    const LevelGeom& v = g.lv[level];
    int n = 0;
    ORB_HIP(hipDeviceSynchronize());
    ORB_HIP(hipMemcpy(&n, e->d_oct_count + (size_t)frame * kOcStride + level, sizeof(int), hipMemcpyDeviceToHost));
    std::vector<uint32_t> keys(std::max(n, 1));
    ORB_HIP(hipMemcpy(keys.data(), e->d_oct_out + (size_t)frame * g.slots_frame + v.out_offset,
                      (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < cap && xys; ++i) {
        xys[3 * i] = key_x(keys[i]); xys[3 * i + 1] = key_y(keys[i]); xys[3 * i + 2] = key_s(keys[i]);
    }
    return n;
}

}  // extern "C"

int orbgpu_debug_pyramid_emulate(int nfeatures, float scale_factor, int nlevels, int width, int height,
                                 const uint8_t* img, size_t img_step, uint8_t* out, size_t out_bytes, int* info) {
    if (!img || !out || nfeatures <= 0 || nlevels <= 0 || nlevels > kMaxLevels || !(scale_factor > 1.f) ||
        width <= 0 || height <= 0 || img_step < (size_t)width)
        return fail(ORBGPU_ERR_ARG, "invalid emulation arguments");
    orbgpu_extractor e;  // host geometry only: no device buffers are allocated
    e.nfeatures = nfeatures;
    e.scale_factor = scale_factor;
    e.nlevels = nlevels;
    e.ini_th = 20;
    e.min_th = 7;
    e.W = width;
    e.H = height;
    e.max_batch = 1;
    std::vector<int4> ptab;
    std::vector<int2> ytab;
    int rc = build_geometry(&e, ptab, ytab, nullptr);
    if (rc) return rc;
    const Geom& g = e.g;
    size_t need = 0;
    for (int l = 1; l < nlevels; ++l) need += (size_t)g.lv[l].w * g.lv[l].h;
    if (out_bytes < need) return fail(ORBGPU_ERR_CAPACITY, "out_bytes smaller than levels 1..L-1");
    std::vector<std::vector<uint8_t>> levels;
    rc = emulate_pyramid(g, ytab, e.pyr_plan, img, img_step, levels);
    if (rc) return rc;
    for (int l = 1; l < nlevels; ++l) {
        std::memcpy(out, levels[(size_t)l].data(), levels[(size_t)l].size());
        out += levels[(size_t)l].size();
    }
    if (info) {
        const int v[8] = {g.tk_ticks, g.tk_t0, g.tk_cwaves, g.tk_pwaves, g.tk_np, g.tk_e, g.tk_lds_bytes,
                          g.lv[0].tk_ring_rows};
        std::memcpy(info, v, sizeof(v));
    }
    return ORBGPU_OK;
}

// The fused pyramid plan's work per tick (tools/pyr_plan_cost.py): rows[k *
// lanes + i] = the rows lane i (entry 0, then entry 1 at i + CL) computes at
// tick k; lane_info[i] = level | tail << 8 (level 0: an idle lane); dims =
// {ticks, lanes, compute waves, entries per lane}.
extern "C" int orbgpu_debug_pyramid_plan_rows(int nfeatures, float scale_factor, int nlevels, int width, int height,
                                              int* rows, size_t rows_n, int* lane_info, size_t lanes_n, int* dims) {
    if (!dims || nfeatures <= 0 || nlevels < 2 || nlevels > kMaxLevels || !(scale_factor > 1.f) || width <= 0 ||
        height <= 0)
        return fail(ORBGPU_ERR_ARG, "invalid plan arguments");
    orbgpu_extractor e;
    e.nfeatures = nfeatures;
    e.scale_factor = scale_factor;
    e.nlevels = nlevels;
    e.ini_th = 20;
    e.min_th = 7;
    e.W = width;
    e.H = height;
    e.max_batch = 1;
    std::vector<int4> ptab;
    std::vector<int2> ytab;
    int rc = build_geometry(&e, ptab, ytab, nullptr);
    if (rc) return rc;
    const Geom& g = e.g;
    const int K = g.tk_ticks, CL = 64 * g.tk_cwaves, E = g.tk_e, n = CL * E;
    dims[0] = K;
    dims[1] = n;
    dims[2] = g.tk_cwaves;
    dims[3] = E;
    if (!rows || !lane_info) return ORBGPU_OK;
    if (rows_n < (size_t)K * n || lanes_n < (size_t)n) return fail(ORBGPU_ERR_CAPACITY, "plan output too small");
    const uint32_t* rng = reinterpret_cast<const uint32_t*>(e.pyr_plan.tab.data()) + g.tk_rng;
    for (int i = 0; i < n; ++i) {
        const int4* r = &e.pyr_plan.ent[(size_t)i * 9];
        lane_info[i] = r[2].w | (r[0].y ? 1 << 8 : 0);
        for (int k = 0; k < K; ++k) rows[(size_t)k * n + i] = (int)((rng[(size_t)k * g.tk_rs + r[0].x] >> 11) & 31u);
    }
    return ORBGPU_OK;
}

namespace {

// StereoArgs common to both entry points: level sizes and scales, thresholds,
// and the level bases of the left / right image of pair 0 (lb0 / rb0: level 0
// from the caller's image pointers, levels >= 1 from the extractors' pyramids)
void stereo_args(const orbgpu_extractor* left, const orbgpu_extractor* right, int lframe, int rframe,
                 const uint8_t* l0, const uint8_t* r0, size_t row_step, size_t pair_step0, int cap, float bf,
                 float min_z, StereoArgs& a) {
    const Geom& g = left->g;
    std::memset(&a, 0, sizeof(a));
    for (int l = 0; l < g.nlevels; ++l) {
        if (l == 0) {
            a.lvl_base[0] = l0;
            a.lvl_base_r[0] = r0;
            a.lvl_pair[0] = pair_step0;
            a.lvl_pitch[0] = (int)row_step;
        } else {
            a.lvl_base[l] = left->d_pyr + g.lv[l].offset + (size_t)lframe * g.lv[l].frame_bytes;
            a.lvl_base_r[l] = right->d_pyr + g.lv[l].offset + (size_t)rframe * g.lv[l].frame_bytes;
            a.lvl_pair[l] = 2 * g.lv[l].frame_bytes;
            a.lvl_pitch[l] = g.lv[l].pitch;
        }
        a.lvl_w[l] = g.lv[l].w;
        a.lvl_h[l] = g.lv[l].h;
        a.scale[l] = left->scale[l];
        a.inv_scale[l] = left->inv_scale[l];
    }
    a.cap = cap;
    a.bf = bf;
    a.max_d = bf / min_z;  // +inf for min_z = 0, as the reference (Frame.cpp:581)
    a.th_orb = (100 + 50) / 2;
    a.rr = (int)std::ceil(2.0f * left->scale[g.nlevels - 1]) + 1;
}

}  // namespace

// Frame::ComputeStereoMatches (Frame.cpp:540-748) over the last extraction.
int orbgpu_stereo_matches_batch_device(orbgpu_extractor* e, const uint8_t* d_images, size_t row_step,
                                       size_t frame_step, int npairs, const orbgpu_keypoint* d_kps,
                                       const uint8_t* d_desc, const int* d_counts, int kp_capacity, float bf,
                                       float min_z, float* d_uright, float* d_depth, void* stream) {
    if (!e || !d_images || !d_kps || !d_desc || !d_counts || !d_uright || !d_depth)
        return fail(ORBGPU_ERR_ARG, "NULL argument");
    DeviceScope ds_(e->device);
    if (npairs < 0 || 2 * npairs > e->max_batch) return fail(ORBGPU_ERR_ARG, "npairs exceeds max_batch / 2");
    if (kp_capacity < e->max_kps || kp_capacity > 65535)
        return fail(ORBGPU_ERR_ARG, "kp_capacity must be >= max_keypoints and < 65536");
    const Geom& g = e->g;
    if (stereo_lds_bytes(kp_capacity, g.lv[0].h) > 160 * 1024)
        return fail(ORBGPU_ERR_UNSUPPORTED, "stereo LDS tables exceed 160 KiB");
    StereoArgs a;
    stereo_args(e, e, 0, 1, d_images, d_images + frame_step, row_step, 2 * frame_step, kp_capacity, bf, min_z, a);
    a.kps = d_kps;
    a.desc = d_desc;
    a.counts = d_counts;
    a.uright = d_uright;
    a.depth = d_depth;
    const size_t nsad = (size_t)npairs * kp_capacity;
    const hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
    {
        std::lock_guard<std::mutex> lk(e->stereo_mu);
        orbgpu_extractor::SadScratch* sc = nullptr;
        for (auto& x : e->stereo_sad)
            if (x.stream == hs) sc = &x;
        if (!sc) {
            e->stereo_sad.push_back({hs, nullptr, 0});
            sc = &e->stereo_sad.back();
        }
        if (nsad > sc->n) {
            if (sc->d) ORB_HIP(hipFree(sc->d));
            sc->d = nullptr;
            sc->n = 0;
            ORB_HIP(hipMalloc((void**)&sc->d, nsad * sizeof(int)));
            sc->n = nsad;
        }
        a.sad = sc->d;
    }
    ORB_HIP(launch_stereo(a, npairs, hs));
    return ORBGPU_OK;
}

// ComputeStereoMatches of a stereo Frame built by two extractors
// (Frame.cpp:84-98): the pyramids of their last orbgpu_extract calls, read in
// place in HBM; keypoints / descriptors from the host.
int orbgpu_stereo_matches_pair(orbgpu_extractor* left, orbgpu_extractor* right, const orbgpu_keypoint* kps_l,
                               const uint8_t* desc_l, int n_l, const orbgpu_keypoint* kps_r, const uint8_t* desc_r,
                               int n_r, float bf, float min_z, float* uright, float* depth) {
    if (!left || !right || n_l < 0 || n_r < 0 || (n_l > 0 && (!kps_l || !desc_l || !uright || !depth)) ||
        (n_r > 0 && (!kps_r || !desc_r)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    DeviceScope ds_(left->device);
    if (left->W != right->W || left->H != right->H || left->nlevels != right->nlevels ||
        left->scale_factor != right->scale_factor)
        return fail(ORBGPU_ERR_ARG, "left and right extractors differ in geometry");
    if (!left->last_img || !right->last_img || left->last_batch < 1 || right->last_batch < 1)
        return fail(ORBGPU_ERR_ARG, "both extractors need an extraction first");
    if (left->last_row != right->last_row) return fail(ORBGPU_ERR_ARG, "level-0 row steps differ");
    // frame capacity a multiple of 64, so the staged L and R arrays are contiguous (28 * 64 and
    // 32 * 64 bytes are multiples of the arena's 256-byte granule): frame f at + f * cap
    const int cap = (std::max(std::max(n_l, n_r), 1) + 63) / 64 * 64;
    if (cap > 65535) return fail(ORBGPU_ERR_ARG, "more than 65535 keypoints");
    if (stereo_lds_bytes(cap, left->g.lv[0].h) > 160 * 1024)
        return fail(ORBGPU_ERR_UNSUPPORTED, "stereo LDS tables exceed 160 KiB");
    if (n_l == 0) return ORBGPU_OK;
    int rc = check_device();
    if (rc) return rc;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    // the pyramids were written on the extractors' streams (orbgpu_extract returned after
    // synchronising them), so the thread's stream may read them directly
    HostCall call(*ctx);
    orbgpu_keypoint *dk, *dk_r;
    uint8_t *dd, *dd_r;
    int* dn;
    float *du, *dz;
    int* ds;
    const int counts[2] = {n_l, n_r};
    rc = call.run([&](HostCall& A) {
        dk = A.inout(kps_l, (size_t)n_l, (size_t)cap);
        dk_r = A.inout(kps_r, (size_t)n_r, (size_t)cap);
        dd = A.inout(desc_l, 32 * (size_t)n_l, 32 * (size_t)cap);
        dd_r = A.inout(desc_r, 32 * (size_t)n_r, 32 * (size_t)cap);
        dn = A.in(counts, 2);
        du = A.out<float>((size_t)cap);
        dz = A.out<float>((size_t)cap);
        ds = A.out<int>((size_t)cap);
    });
    if (rc) return rc;
    if (dk_r != dk + cap || dd_r != dd + 32 * (size_t)cap) return fail(ORBGPU_ERR_ARG, "internal: staging layout");
    StereoArgs a;
    stereo_args(left, right, 0, 0, left->last_img, right->last_img, left->last_row, 0, cap, bf, min_z, a);
    a.kps = dk;
    a.desc = dd;
    a.counts = dn;
    a.uright = du;
    a.depth = dz;
    a.sad = ds;
    ORB_HIP(launch_stereo(a, 1, ctx->stream));
    call.fetch(du, uright, 4 * (size_t)n_l);
    call.fetch(dz, depth, 4 * (size_t)n_l);
    return call.finish();
}
