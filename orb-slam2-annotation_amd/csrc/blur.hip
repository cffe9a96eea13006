// blur.hip -- GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) of every
// pyramid level (ORBextractor.cpp:1097-1098) with OpenCV-2.4's 8U
// arithmetic: integer kernel [18,34,49,55,49,34,18] (x256), exact int32 row
// pass, column pass rounded half-to-even on x < 4*floor(w/4) (the SSE2
// float path of SymmColumnVec_32s8u) and half-up on the scalar tail
// (FixedPtCastEx<int,uchar>, 16 bits).
//
// One launch over all levels of all frames: 256-thread blocks own a 64x32
// output tile, stage the 70x38 input (REFLECT_101 on the image border) in
// LDS, run the row pass into LDS and write 4 output bytes per thread-step.
// Roofline: HBM streaming (read + write each level once).
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

constexpr int TW = 64, TH = 32, R = 3;
constexpr int IW = TW + 2 * R, IH = TH + 2 * R;  // 70 x 38
__constant__ int c_bk[7] = {18, 34, 49, 55, 49, 34, 18};

__device__ inline int reflect101(int p, int n) {
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__global__ __launch_bounds__(256) void blur_levels_kernel(Geom g, const uint8_t* __restrict__ img0, size_t row0,
                                                          size_t frame0, const uint8_t* __restrict__ pyr,
                                                          uint8_t* __restrict__ blur) {
    __shared__ uint8_t s_in[IH * 72];
    __shared__ uint16_t s_row[IH * TW];
    const int f = blockIdx.y;
    const int t = blockIdx.x;
    int l = 0;
    while (l + 1 < g.nlevels && t >= g.lv[l + 1].blur_tile_base) ++l;
    const LevelGeom& L = g.lv[l];
    const int tt = t - L.blur_tile_base;
    const int ty = tt / L.blur_tiles_x, tx = tt - ty * L.blur_tiles_x;
    const int x0 = tx * TW, y0 = ty * TH;
    const uint8_t* src = l == 0 ? img0 + (size_t)f * frame0 : pyr + L.offset + (size_t)f * L.frame_bytes;
    const size_t sp = l == 0 ? row0 : (size_t)L.pitch;
    uint8_t* dst = blur + L.blur_offset + (size_t)f * L.blur_frame_bytes;

    for (int idx = threadIdx.x; idx < IW * IH; idx += 256) {
        const int r = idx / IW, c = idx - r * IW;
        const int yy = reflect101(y0 - R + r, L.h), xx = reflect101(x0 - R + c, L.w);
        s_in[r * 72 + c] = src[(size_t)yy * sp + xx];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < IH * TW; idx += 256) {
        const int r = idx / TW, c = idx - r * TW;
        const uint8_t* p = s_in + r * 72 + c;
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 7; ++j) acc += c_bk[j] * p[j];
        s_row[r * TW + c] = (uint16_t)acc;
    }
    __syncthreads();
    const int w4 = L.w & ~3;
    for (int idx = threadIdx.x; idx < TH * (TW / 4); idx += 256) {
        const int r = idx / (TW / 4), c4 = (idx - r * (TW / 4)) * 4;
        const int y = y0 + r;
        if (y >= L.h) continue;
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = c4 + k;
            int v = 0;
#pragma unroll
            for (int i = 0; i < 7; ++i) v += c_bk[i] * (int)s_row[(r + i) * TW + c];
            const int x = x0 + c;
            int o;
            if (x < w4) {
                const int q = v >> 16, rem = v & 0xFFFF;
                o = q + ((rem > 32768) | ((rem == 32768) & (q & 1)));
            } else {
                o = (v + 32768) >> 16;
            }
            packed |= (uint32_t)min(o, 255) << (8 * k);
        }
        const int x = x0 + c4;
        uint8_t* d = dst + (size_t)y * L.pitch + x;
        if (x + 3 < L.pitch) {
            *reinterpret_cast<uint32_t*>(d) = packed;  // pitch is a multiple of 16
        }
    }
}

}  // namespace

hipError_t launch_blur_levels(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                              const uint8_t* pyr, uint8_t* blur, hipStream_t stream) {
    dim3 grid(g.blur_tiles_frame, batch);
    hipLaunchKernelGGL(blur_levels_kernel, grid, dim3(256), 0, stream, g, img0, row0, frame0, pyr, blur);
    return hipGetLastError();
}

}  // namespace orbgpu
