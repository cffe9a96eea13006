// blur.hip -- GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) of every
// pyramid level (ORBextractor.cpp:1097-1098) with OpenCV-2.4's 8U
// arithmetic: integer kernel [18,34,49,55,49,34,18] (x256), exact int32 row
// pass, column pass rounded half-to-even on x < 4*floor(w/4) (the SSE2
// float path of SymmColumnVec_32s8u) and half-up on the scalar tail
// (FixedPtCastEx<int,uchar>, 16 bits).
//
// One launch over all levels of all frames; a thread owns 4 columns x 63
// rows (see below).  Bound: VALU (packed u16 row pass, packed f32 column
// pass); HBM: read + write each level once, 6/63 halo rows re-read from L2.
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "blur_device.h"

namespace orbgpu {

namespace {

constexpr int kStrip = kBlurStrip;
using namespace blurdev;

// BORDER_REFLECT_101 for an overshoot of at most n - 1 (<= 6 for the filter
// taps; the interior strip's unused prefetches go up to 9 rows past a strip
// and are clamped after reflection)
__device__ inline int reflect101(int p, int n) { return p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p); }

// Interior strip (columns x0-3 .. x0+6 need no reflection): rows [y0, y1)
// in groups of 7.  Row slot u of a group is consumed and immediately
// refilled with the row 7 ahead, so 7 rows of loads are in flight and the
// slots never move between registers (no copy waits on a pending load).
// Rows past the level reflect (BORDER_REFLECT_101); prefetches past what the
// strip needs are clamped to the last row and unused.
__device__ __forceinline__ void blur_strip_interior(const uint8_t* __restrict__ src, uint32_t sp, int H, int x0,
                                                    int y0, int y1, bool simd, uint8_t* __restrict__ dst,
                                                    uint32_t dp) {
    const uint8_t* base = src + x0;
    auto fetch = [&](int yy) {
        const int r = min(reflect101(yy, H), H - 1);
        const uint8_t* row = base + __umul24((uint32_t)r, sp);
        Raw3 R;
        R.a = *reinterpret_cast<const uint32_t*>(row - 4);
        R.b = *reinterpret_cast<const uint32_t*>(row);
        R.c = *reinterpret_cast<const uint32_t*>(row + 4);
        return R;
    };
    f32x2 wl[7], wh[7];  // row-pass window: slot (y - y0 + i) % 7 holds row y - 3 + i
#pragma unroll
    for (int i = 0; i < 6; ++i) row_pass_raw(fetch(y0 - 3 + i), wl[i], wh[i]);
    Raw3 raw[7];  // raw[u] = row y + u + 3 of the current group
#pragma unroll
    for (int u = 0; u < 7; ++u) raw[u] = fetch(y0 + 3 + u);
    for (int y = y0; y < y1; y += 7) {
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            row_pass_raw(raw[u], wl[(u + 6) % 7], wh[(u + 6) % 7]);
            raw[u] = fetch(y + u + 10);
            const f32x2 lo = col_pass(wl[u % 7], wl[(u + 1) % 7], wl[(u + 2) % 7], wl[(u + 3) % 7], wl[(u + 4) % 7],
                                      wl[(u + 5) % 7], wl[(u + 6) % 7]);
            const f32x2 hi = col_pass(wh[u % 7], wh[(u + 1) % 7], wh[(u + 2) % 7], wh[(u + 3) % 7], wh[(u + 4) % 7],
                                      wh[(u + 5) % 7], wh[(u + 6) % 7]);
            if (y + u < y1) *reinterpret_cast<uint32_t*>(dst + __umul24((uint32_t)(y + u), dp) + x0) = pack4(lo, hi, simd);
        }
    }
}

// Edge strip (some of columns x0-3 .. x0+6 reflect): byte loads.
__device__ __noinline__ void blur_strip_edge(const uint8_t* __restrict__ src, uint32_t sp, int W, int H, int x0, int y0,
                                             int y1, bool simd, uint8_t* __restrict__ dst, uint32_t dp) {
    auto filter_row = [&](int yy, f32x2& lo, f32x2& hi) {
        const uint8_t* row = src + __umul24((uint32_t)reflect101(yy, H), sp);
        int px[10];
#pragma unroll
        for (int j = 0; j < 10; ++j) px[j] = row[reflect101(x0 - 3 + j, W)];
        uint32_t P[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) P[j] = (uint32_t)px[j] | ((uint32_t)px[j + 1] << 16);
        row_pass(P, lo, hi);
    };
    f32x2 wl[7], wh[7];
#pragma unroll
    for (int i = 0; i < 6; ++i) filter_row(y0 - 3 + i, wl[i], wh[i]);
    for (int y = y0; y < y1; y += 7) {
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            filter_row(y + u + 3, wl[(u + 6) % 7], wh[(u + 6) % 7]);
            const f32x2 lo = col_pass(wl[u % 7], wl[(u + 1) % 7], wl[(u + 2) % 7], wl[(u + 3) % 7], wl[(u + 4) % 7],
                                      wl[(u + 5) % 7], wl[(u + 6) % 7]);
            const f32x2 hi = col_pass(wh[u % 7], wh[(u + 1) % 7], wh[(u + 2) % 7], wh[(u + 3) % 7], wh[(u + 4) % 7],
                                      wh[(u + 5) % 7], wh[(u + 6) % 7]);
            if (y + u < y1) *reinterpret_cast<uint32_t*>(dst + __umul24((uint32_t)(y + u), dp) + x0) = pack4(lo, hi, simd);
        }
    }
}

// One thread = 4 adjacent output columns x a 63-row strip of one level.
// Walking down the strip it keeps the last 7 row-pass results (as floats)
// in registers -- the window rotates statically (the row loop is unrolled
// by 7) -- so every input row is read once per strip (+6 halo rows).
__global__ __launch_bounds__(256) void blur_levels_kernel(Geom g, int tile0, int items_frame, int items_total,
                                                          const uint8_t* __restrict__ img0, size_t row0,
                                                          size_t frame0, const uint8_t* __restrict__ pyr,
                                                          uint8_t* __restrict__ blur) {
    const int item = blockIdx.x * 256 + threadIdx.x;
    if (item >= items_total) return;
    const int f = item / items_frame;
    const int it = tile0 + item - f * items_frame;  // tile of the frame (levels from tile0's)
    int l = 0;
    while (l + 1 < g.nlevels && it >= g.lv[l + 1].blur_tile_base) ++l;
    const LevelGeom& L = g.lv[l];
    const int k = it - L.blur_tile_base;
    const int strip = k / L.blur_tiles_x, q = k - strip * L.blur_tiles_x;
    const int x0 = 4 * q, y0 = strip * kStrip;
    const int y1 = min(y0 + kStrip, L.h);
    const uint8_t* src = l == 0 ? img0 + (size_t)f * frame0 : pyr + L.offset + (size_t)f * L.frame_bytes;
    const size_t sp = l == 0 ? row0 : (size_t)L.pitch;
    uint8_t* dst = blur + L.blur_offset + (size_t)f * L.blur_frame_bytes;
    const bool simd = x0 < (L.w & ~3);  // all 4 columns on the vector path, else all on the tail
    if (x0 >= 4 && x0 + 7 < L.w)
        blur_strip_interior(src, (uint32_t)sp, L.h, x0, y0, y1, simd, dst, (uint32_t)L.pitch);
    else
        blur_strip_edge(src, (uint32_t)sp, L.w, L.h, x0, y0, y1, simd, dst, (uint32_t)L.pitch);
}

}  // namespace

hipError_t launch_blur_levels(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                              const uint8_t* pyr, uint8_t* blur, hipStream_t stream, int level_from) {
    if (level_from >= g.nlevels) return hipSuccess;
    const int tile0 = level_from > 0 ? g.lv[level_from].blur_tile_base : 0;
    const int per_frame = g.blur_tiles_frame - tile0;
    const int items = per_frame * batch;
    hipLaunchKernelGGL(blur_levels_kernel, dim3((items + 255) / 256), dim3(256), 0, stream, g, tile0, per_frame,
                       items, img0, row0, frame0, pyr, blur);
    return hipGetLastError();
}

}  // namespace orbgpu
