// pyramid.hip -- ORBextractor::ComputePyramid (ORBextractor.cpp:1123-1148):
// level l = resize(level l-1, INTER_LINEAR) with OpenCV-2.4's 8U fixed-point
// arithmetic (Q11 horizontal taps, VResizeLinearVec_32s8u vertical SIMD
// rounding on x < simd_end, FixedPtCast<int,uchar,22> on the tail).
// The per-level x/y tap tables are precomputed on the host (orbgpu.cpp,
// build_resize_tables) exactly like resize() builds xofs/ialpha/yofs/ibeta.
//
// Roofline: HBM-bound streaming; algorithmic bytes per level = |P_{l-1}| read
// + |P_l| written.  One launch per level over the whole batch (frames on
// blockIdx.z); each block stages the two source rows of its output row band
// through LDS with 16-byte loads, so every source byte is fetched from HBM
// once per output row pair instead of once per tap.
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

constexpr int kPyrRows = 4;           // output rows per block
constexpr int kPyrThreads = 256;
constexpr int kMaxSrcW = 2112;        // staged source row capacity (bytes)

__device__ inline int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

__device__ inline int vres_simd(int h0, int h1, int b0, int b1) {
    const int t0 = sat_s16(h0 >> 4), t1 = sat_s16(h1 >> 4);
    const int m0 = (t0 * b0) >> 16, m1 = (t1 * b1) >> 16;
    const int v = sat_s16(sat_s16(m0 + m1) + 2) >> 2;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

__device__ inline int vres_scalar(int h0, int h1, int b0, int b1) {
    const int v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// One block = kPyrRows output rows x the full output width of one frame.
// Source rows needed by the band are staged in LDS (they are contiguous:
// at most kPyrRows+2 distinct rows for a 1/1.2 downscale).
__global__ __launch_bounds__(kPyrThreads) void pyr_level_kernel(
    const uint8_t* __restrict__ src, int src_pitch, size_t src_frame, int sw, int sh,
    uint8_t* __restrict__ dst, int dst_pitch, size_t dst_frame, int dw, int dh, int simd_end,
    const int2* __restrict__ xtab, const int2* __restrict__ ytab) {
    __shared__ __attribute__((aligned(16))) uint8_t s_src[(kPyrRows + 3) * kMaxSrcW];
    const int f = blockIdx.z;
    const int dy0 = blockIdx.x * kPyrRows;
    const uint8_t* S = src + (size_t)f * src_frame;
    // rows touched by this band: [ylo, yhi]
    const int dyl = min(dy0 + kPyrRows, dh) - 1;
    const int ylo = ytab[dy0].x & 0xFFFF;
    const int yhi = ytab[dyl].x >> 16;
    const int nrows = yhi - ylo + 1;  // <= kPyrRows + 3 (checked on host)
    // stage rows with 16-byte loads (pitch is a multiple of 16 for levels >= 1,
    // and the input row step is checked to be a multiple of 16 on the host)
    const int vec_per_row = (sw + 15) >> 4;
    for (int idx = threadIdx.x; idx < nrows * vec_per_row; idx += kPyrThreads) {
        const int r = idx / vec_per_row, v = idx - r * vec_per_row;
        const uint4 q = *reinterpret_cast<const uint4*>(S + (size_t)(ylo + r) * src_pitch + v * 16);
        *reinterpret_cast<uint4*>(s_src + r * kMaxSrcW + v * 16) = q;
    }
    __syncthreads();
    // each thread: 4 consecutive output pixels of one row
    const int quads = (dw + 3) >> 2;
    for (int idx = threadIdx.x; idx < kPyrRows * quads; idx += kPyrThreads) {
        const int r = idx / quads, qx = idx - r * quads;
        const int dy = dy0 + r;
        if (dy >= dh) break;
        const int2 yt = ytab[dy];
        const uint8_t* r0 = s_src + ((yt.x & 0xFFFF) - ylo) * kMaxSrcW;
        const uint8_t* r1 = s_src + ((yt.x >> 16) - ylo) * kMaxSrcW;
        const int b0 = (int)(short)(yt.y & 0xFFFF), b1 = yt.y >> 16;
        uint32_t out = 0;
        const int dx0 = qx * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int dx = dx0 + k;
            if (dx < dw) {
                const int2 xt = xtab[dx];
                const int sx0 = xt.x & 0xFFFF, sx1 = xt.x >> 16;
                const int a0 = (int)(short)(xt.y & 0xFFFF), a1 = xt.y >> 16;
                const int h0 = r0[sx0] * a0 + r0[sx1] * a1;
                const int h1 = r1[sx0] * a0 + r1[sx1] * a1;
                const int v = dx < simd_end ? vres_simd(h0, h1, b0, b1) : vres_scalar(h0, h1, b0, b1);
                out |= (uint32_t)v << (8 * k);
            }
        }
        uint8_t* D = dst + (size_t)f * dst_frame + (size_t)dy * dst_pitch + dx0;
        // dst pitch is padded to 16 bytes, so a full 4-byte store is in bounds
        *reinterpret_cast<uint32_t*>(D) = out;
    }
}

}  // namespace

int pyr_max_src_width() { return kMaxSrcW; }
int pyr_rows_per_block() { return kPyrRows; }

hipError_t launch_pyramid_level(const uint8_t* src, int src_pitch, size_t src_frame, int sw, int sh,
                                uint8_t* dst, int dst_pitch, size_t dst_frame, int dw, int dh,
                                int simd_end, const int2* xtab, const int2* ytab, int batch,
                                hipStream_t stream) {
    dim3 grid((dh + kPyrRows - 1) / kPyrRows, 1, batch);
    hipLaunchKernelGGL(pyr_level_kernel, grid, dim3(kPyrThreads), 0, stream, src, src_pitch, src_frame,
                       sw, sh, dst, dst_pitch, dst_frame, dw, dh, simd_end, xtab, ytab);
    return hipGetLastError();
}

}  // namespace orbgpu
