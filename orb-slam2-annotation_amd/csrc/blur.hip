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

namespace orbgpu {

namespace {

constexpr int kStrip = kBlurStrip;

// BORDER_REFLECT_101 for an overshoot of at most n - 1 (<= 6 for the filter
// taps; the interior strip's unused prefetches go up to 9 rows past a strip
// and are clamped after reflection)
__device__ inline int reflect101(int p, int n) { return p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p); }

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Row pass of 4 adjacent columns: packed 16-bit arithmetic, two columns per
// register.  P[j] = (px[j], px[j+1]) with px[j] = column x0 - 3 + j.  The
// symmetric sum 18(a+g) + 34(b+f) + 49(c+e) + 55d of 8-bit inputs is at most
// 255 * 257 = 65535: exact in u16.  Returns the 4 sums as floats (exact).
__device__ __forceinline__ void row_pass(const uint32_t (&P)[9], f32x2& lo, f32x2& hi) {
    const u16x2* Q = reinterpret_cast<const u16x2*>(P);
    const u16x2 k18 = {18, 18}, k34 = {34, 34}, k49 = {49, 49}, k55 = {55, 55};
    const u16x2 r01 = (Q[0] + Q[6]) * k18 + (Q[1] + Q[5]) * k34 + (Q[2] + Q[4]) * k49 + Q[3] * k55;
    const u16x2 r23 = (Q[2] + Q[8]) * k18 + (Q[3] + Q[7]) * k34 + (Q[4] + Q[6]) * k49 + Q[5] * k55;
    lo = f32x2{(float)r01.x, (float)r01.y};
    hi = f32x2{(float)r23.x, (float)r23.y};
}

// Column pass over the 7-row window (w[i] = row y - 3 + i), two columns per
// packed-f32 op.  Every product and partial sum is an integer below 2^24
// unless the total is (then the result saturates to 255 either way), so the
// float arithmetic is exact.
__device__ __forceinline__ f32x2 col_pass(f32x2 w0, f32x2 w1, f32x2 w2, f32x2 w3, f32x2 w4, f32x2 w5, f32x2 w6) {
    const f32x2 k18 = {18.f, 18.f}, k34 = {34.f, 34.f}, k49 = {49.f, 49.f}, k55 = {55.f, 55.f};
    f32x2 s = w3 * k55;
    s = __builtin_elementwise_fma(w2 + w4, k49, s);
    s = __builtin_elementwise_fma(w1 + w5, k34, s);
    s = __builtin_elementwise_fma(w0 + w6, k18, s);
    return s * f32x2{1.f / 65536.f, 1.f / 65536.f};  // exact: power of two
}

// 8-bit result of one column on the scalar tail (x >= 4*floor(w/4)):
// FixedPtCastEx rounds half up.  (The vector path, SymmColumnVec_32s8u,
// rounds half to even: v_cvt_pk_u8_f32 in store_row.)
__device__ __forceinline__ uint32_t to_u8(float v) {
    return (uint32_t)fminf(__builtin_floorf(v + 0.5f), 255.f);  // v + 0.5 exact (< 2^8, 16 frac bits)
}

// 8-bit packing of 4 filtered columns; v_cvt_pk_u8_f32 rounds to nearest
// even and saturates (the vector path), to_u8 rounds half up (the tail).
__device__ __forceinline__ uint32_t pack4(f32x2 lo, f32x2 hi, bool simd) {
    if (simd) {
        uint32_t packed = __builtin_amdgcn_cvt_pk_u8_f32(lo.x, 0, 0u);
        packed = __builtin_amdgcn_cvt_pk_u8_f32(lo.y, 1, packed);
        packed = __builtin_amdgcn_cvt_pk_u8_f32(hi.x, 2, packed);
        return __builtin_amdgcn_cvt_pk_u8_f32(hi.y, 3, packed);
    }
    return to_u8(lo.x) | (to_u8(lo.y) << 8) | (to_u8(hi.x) << 16) | (to_u8(hi.y) << 24);
}

#ifndef BLUR_PROBE
#define BLUR_PROBE 0  // diagnostic builds only: bit 0 = no stores in interior strips
#endif

struct Raw3 {
    uint32_t a, b, c;  // level columns x0-4 .. x0+7
};

__device__ __forceinline__ void row_pass_raw(const Raw3& R, f32x2& lo, f32x2& hi) {
    uint32_t P[9];
    // bytes of (b:a) / (c:b) as v_perm_b32 sees them: low word 0-3, high word 4-7
    P[0] = __builtin_amdgcn_perm(R.b, R.a, 0x0c020c01u);
    P[1] = __builtin_amdgcn_perm(R.b, R.a, 0x0c030c02u);
    P[2] = __builtin_amdgcn_perm(R.b, R.a, 0x0c040c03u);
    P[3] = __builtin_amdgcn_perm(R.b, R.a, 0x0c050c04u);
    P[4] = __builtin_amdgcn_perm(R.c, R.b, 0x0c020c01u);
    P[5] = __builtin_amdgcn_perm(R.c, R.b, 0x0c030c02u);
    P[6] = __builtin_amdgcn_perm(R.c, R.b, 0x0c040c03u);
    P[7] = __builtin_amdgcn_perm(R.c, R.b, 0x0c050c04u);
    P[8] = __builtin_amdgcn_perm(R.c, R.b, 0x0c060c05u);
    row_pass(P, lo, hi);
}

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
#if BLUR_PROBE & 2
        R.a = (uint32_t)(uintptr_t)row * 0x9E3779B1u;  // timing probe: no loads
        R.b = R.a ^ 0x5bd1e995u;
        R.c = R.a + 0x1b873593u;
#else
        R.a = *reinterpret_cast<const uint32_t*>(row - 4);
        R.b = *reinterpret_cast<const uint32_t*>(row);
        R.c = *reinterpret_cast<const uint32_t*>(row + 4);
#endif
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
#if BLUR_PROBE & 1
            if (y + u < y1 && pack4(lo, hi, simd) == 0x12345678u) *reinterpret_cast<uint32_t*>(dst) = 0;  // timing probe: no stores
#else
            if (y + u < y1) *reinterpret_cast<uint32_t*>(dst + __umul24((uint32_t)(y + u), dp) + x0) = pack4(lo, hi, simd);
#endif
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
#ifndef BLUR_WAVES_PER_EU
#define BLUR_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(256, BLUR_WAVES_PER_EU) void blur_levels_kernel(Geom g, int items_frame, int items_total,
                                                          const uint8_t* __restrict__ img0, size_t row0,
                                                          size_t frame0, const uint8_t* __restrict__ pyr,
                                                          uint8_t* __restrict__ blur) {
    const int item = blockIdx.x * 256 + threadIdx.x;
    if (item >= items_total) return;
    const int f = item / items_frame;
    const int it = item - f * items_frame;
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
                              const uint8_t* pyr, uint8_t* blur, hipStream_t stream) {
    const int items = g.blur_tiles_frame * batch;
    hipLaunchKernelGGL(blur_levels_kernel, dim3((items + 255) / 256), dim3(256), 0, stream, g, g.blur_tiles_frame,
                       items, img0, row0, frame0, pyr, blur);
    return hipGetLastError();
}

}  // namespace orbgpu
