// blur.hip -- GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) of every
// pyramid level (ORBextractor.cpp:1097-1098) with OpenCV-2.4's 8U
// arithmetic: integer kernel [18,34,49,55,49,34,18] (x256), exact int32 row
// pass, column pass rounded half-to-even on x < 4*floor(w/4) (the SSE2
// float path of SymmColumnVec_32s8u) and half-up on the scalar tail
// (FixedPtCastEx<int,uchar>, 16 bits).
//
// One launch over all levels of all frames; a thread owns 4 columns x 64
// rows (see below).  Roofline: HBM streaming (read + write each level once,
// 6/64 halo rows re-read from L2).
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

constexpr int kStrip = 64;  // output rows per thread
__constant__ int c_bk[7] = {18, 34, 49, 55, 49, 34, 18};

__device__ inline int reflect101(int p, int n) {
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

// One thread = 4 adjacent output columns x a 64-row strip of one level.
// Walking down the strip it keeps the last 7 row-pass results in registers
// (separable filter as a sliding window), so every input row is read once
// per strip (+6 halo rows) with three aligned dword loads.
__global__ __launch_bounds__(256) void blur_levels_kernel(Geom g, int items_frame, int items_total,
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
    const bool interior = x0 >= 4 && x0 + 7 < L.w;  // columns x0-3 .. x0+6 need no reflection
    const int w4 = L.w & ~3;

    int rp[7][4];  // row-pass sliding window, rows y-3 .. y+3
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) rp[i][c] = 0;
    for (int yy = y0 - 3; yy < y1 + 3; ++yy) {
        const uint8_t* row = src + (size_t)reflect101(yy, L.h) * sp;
        int px[10];  // level columns x0-3 .. x0+6
        if (interior) {
            const uint32_t a = *reinterpret_cast<const uint32_t*>(row + x0 - 4);
            const uint32_t b = *reinterpret_cast<const uint32_t*>(row + x0);
            const uint32_t c = *reinterpret_cast<const uint32_t*>(row + x0 + 4);
            px[0] = (a >> 8) & 255; px[1] = (a >> 16) & 255; px[2] = a >> 24;
            px[3] = b & 255; px[4] = (b >> 8) & 255; px[5] = (b >> 16) & 255; px[6] = b >> 24;
            px[7] = c & 255; px[8] = (c >> 8) & 255; px[9] = (c >> 16) & 255;
        } else {
#pragma unroll
            for (int j = 0; j < 10; ++j) px[j] = row[reflect101(x0 - 3 + j, L.w)];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) rp[i][c] = rp[i + 1][c];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            int acc = 0;
#pragma unroll
            for (int j = 0; j < 7; ++j) acc += c_bk[j] * px[c + j];
            rp[6][c] = acc;
        }
        const int y = yy - 3;
        if (y >= y0) {
            uint32_t packed = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                int v = 0;
#pragma unroll
                for (int i = 0; i < 7; ++i) v += c_bk[i] * rp[i][c];
                int o;
                if (x0 + c < w4) {  // SymmColumnVec_32s8u: float path, round half to even
                    const int qq = v >> 16, rem = v & 0xFFFF;
                    o = qq + ((rem > 32768) | ((rem == 32768) & (qq & 1)));
                } else {            // scalar tail: FixedPtCastEx, round half up
                    o = (v + 32768) >> 16;
                }
                packed |= (uint32_t)min(o, 255) << (8 * c);
            }
            *reinterpret_cast<uint32_t*>(dst + (size_t)y * L.pitch + x0) = packed;  // x0+3 < pitch
        }
    }
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
