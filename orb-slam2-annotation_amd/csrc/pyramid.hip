// pyramid.hip -- ORBextractor::ComputePyramid (ORBextractor.cpp:1123-1148)
// for all levels of a frame band in ONE launch.
//
// Level l = resize(level l-1, INTER_LINEAR) with OpenCV-2.4's 8U fixed-point
// arithmetic: Q11 horizontal taps (exact int), VResizeLinearVec_32s8u on
// x < simd_end and FixedPtCast<int,uchar,22> on the tail.  The x/y tap
// tables come from the host (orbgpu.cpp, build_resize_tables) exactly as
// resize() builds xofs/ialpha/yofs/ibeta.
//
// Fusion: a block owns one horizontal band of one frame and walks the levels
// bottom-up.  Each level's band rows (its owned rows plus the few halo rows
// the band's next level reads, planned on the host: plan_pyramid_bands) are
// computed from the previous level's rows held in LDS, written to LDS for the
// next level and, for owned rows, to HBM.  The band's level-0 rows are staged
// into LDS once with 16-byte loads.  So every level is written to HBM once and never read back by
// this pass: HBM traffic is |P_0| (+ halo) + sum_l |P_l|, while the
// algorithmic bytes of the reference's level-by-level pass
// (sum_l |P_{l-1}| + |P_l|) are larger.
//
// Per output pixel: two 8-byte windows of the source rows (one dword pair
// each), v_perm_b32 spreads the tap pair into 16-bit lanes and
// v_dot2_u32_u16 applies (ialpha0, ialpha1) -- the exact horizontal sum --
// then the vertical rounding.  No saturation is needed: with non-negative
// Q11 weights summing to 2048 (+-1), every intermediate is in range
// (h <= 255*2048; the SIMD-path sum of the two >>16 products <= 1020).
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

constexpr int kPyrThreads = 1024;

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// One level's band rows [r0, r1).  Thread layout: quad column q of 4 output
// pixels x row group rg walking rows r0+rg, r0+rg+rgroups, ..., so the
// column taps stay in registers for the whole level.  Per quad the taps come
// from ptab (3 x int4: (lo0, wt0, lo1, wt1), (lo2, wt2, lo3, wt3), (sel0..3);
// lo = byte offset of the dword pair holding taps sx and sx+1 -- whenever the
// second tap has a non-zero weight; rows are padded so reading past a row end
// is safe -- sel = the v_perm_b32 selector spreading the two taps into 16-bit
// lanes, wt = (ialpha0, ialpha1)).  s_rows[r - r0] = (LDS offset of source
// row y0, of y1, ibeta0, ibeta1).
__device__ __forceinline__ void resize_band(const uint8_t* __restrict__ lds, const LevelGeom& V, int r0, int r1,
                                            int own0, int own1, const int4* __restrict__ ptab,
                                            const int4* __restrict__ s_rows, uint8_t* __restrict__ lds_dst,
                                            uint8_t* __restrict__ hbm_dst) {
    const int quads = (V.w + 3) >> 2;
    const int rg = (int)__umulhi((uint32_t)threadIdx.x, V.quad_magic);
    const int q = threadIdx.x - rg * quads;
    if (rg >= V.rgroups || r0 + rg >= r1) return;
    const int4 ta = ptab[3 * q], tb = ptab[3 * q + 1], tc = ptab[3 * q + 2];
    const uint8_t* col[4] = {lds + ta.x, lds + ta.z, lds + tb.x, lds + tb.z};
    const uint32_t wt[4] = {(uint32_t)ta.y, (uint32_t)ta.w, (uint32_t)tb.y, (uint32_t)tb.w};
    const uint32_t sel[4] = {(uint32_t)tc.x, (uint32_t)tc.y, (uint32_t)tc.z, (uint32_t)tc.w};
    // all four pixels inside VResizeLinearVec_32s8u's coverage: only the last
    // quad of a row can reach the scalar tail
    const bool all_simd = 4 * q + 3 < V.simd_end;
    uint8_t* ldst = lds_dst ? lds_dst + 4 * q : nullptr;
    uint8_t* hdst = hbm_dst + 4 * q;
    for (int r = r0 + rg; r < r1; r += V.rgroups) {
        const int4 yr = s_rows[r - r0];
        uint32_t h0[4], h1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t* a = reinterpret_cast<const uint32_t*>(col[k] + yr.x);
            const uint32_t* b = reinterpret_cast<const uint32_t*>(col[k] + yr.y);
            const uint32_t p0 = __builtin_amdgcn_perm(a[1], a[0], sel[k]);
            const uint32_t p1 = __builtin_amdgcn_perm(b[1], b[0], sel[k]);
            h0[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p0), __builtin_bit_cast(us2, wt[k]), 0u, false);
            h1[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p1), __builtin_bit_cast(us2, wt[k]), 0u, false);
        }
        uint32_t out = 0;
        if (all_simd) {
            // ((h>>4)*b0 >> 16) + ((h'>>4)*b1 >> 16) + 2, with the +2 folded
            // into the high half of the first product (no carry: < 2^27)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t m0 = __umul24(h0[k] >> 4, (uint32_t)yr.z) + (2u << 16);
                const uint32_t m1 = __umul24(h1[k] >> 4, (uint32_t)yr.w);
                out |= (((m0 >> 16) + (m1 >> 16)) >> 2) << (8 * k);
            }
        } else {  // the last quad of a row: scalar tail for x >= simd_end
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = (int)h0[k], b = (int)h1[k];
                const int v = 4 * q + k < V.simd_end ? ((((a >> 4) * yr.z) >> 16) + (((b >> 4) * yr.w) >> 16) + 2) >> 2
                                                     : (a * yr.z + b * yr.w + (1 << 21)) >> 22;
                out |= (uint32_t)v << (8 * k);
            }
        }
        // bytes past V.w land in the row padding (LDS pitch and HBM pitch are
        // multiples of 4 and 16)
        if (ldst) *reinterpret_cast<uint32_t*>(ldst + (r - r0) * V.lds_pitch) = out;
        if (r >= own0 && r < own1) *reinterpret_cast<uint32_t*>(hdst + r * V.pitch) = out;
    }
}

__global__ __launch_bounds__(kPyrThreads) void pyramid_kernel(Geom g, const int4* __restrict__ bands,
                                                              const int4* __restrict__ ptab,
                                                              const int2* __restrict__ ytab,
                                                              const uint8_t* __restrict__ img0, size_t row0,
                                                              size_t frame0, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_pyr[];
    const int S = g.pyr_bands;
    const int f = blockIdx.x / S;
    const int band = blockIdx.x - f * S;
    const int L = g.nlevels;
    const int4* bt = bands + band * L;
    int4* s_rows = reinterpret_cast<int4*>(s_pyr + g.pyr_lds_y);
    // stage: this band's level-0 rows (16-byte loads; row0 is a multiple of 16)
    // and, per band row of every level, its source rows' LDS offsets and y taps
    {
        const int4 b = bt[0];
        const int v4 = (g.lv[0].w + 15) >> 4;
        const uint8_t* src = img0 + (size_t)f * frame0 + (size_t)b.x * row0;
        uint8_t* dst = s_pyr + g.pyr_lds_b;
        const int n = (b.y - b.x) * v4;
        for (int i = threadIdx.x; i < n; i += kPyrThreads) {
            const int r = (int)__umulhi((uint32_t)i, g.lv[0].quad_magic);
            const int c = i - r * v4;
            *reinterpret_cast<uint4*>(dst + r * g.lv[0].lds_pitch + 16 * c) =
                *reinterpret_cast<const uint4*>(src + (size_t)r * row0 + 16 * c);
        }
        int off = 0;
        for (int l = 1; l < L; ++l) {
            const int4 bl = bt[l];
            const int src_lo = bt[l - 1].x, sp = g.lv[l - 1].lds_pitch;
            const int base = ((l - 1) & 1) ? g.pyr_lds_a : g.pyr_lds_b;
            const int2* yt = ytab + g.lv[l].ytab_offset + bl.x;
            for (int i = threadIdx.x; i < bl.y - bl.x; i += kPyrThreads) {
                const int2 t = yt[i];
                s_rows[off + i] = make_int4(base + ((t.x & 0xFFFF) - src_lo) * sp, base + ((t.x >> 16) - src_lo) * sp,
                                            t.y & 0xFFFF, (int)((uint32_t)t.y >> 16));
            }
            off += bl.y - bl.x;
        }
    }
    __syncthreads();
    int yoff = 0;
    for (int l = 1; l < L; ++l) {
        const LevelGeom& V = g.lv[l];
        const int4 b = bt[l];  // need [x, y), owned [z, w)
        uint8_t* dst_lds = l + 1 < L ? s_pyr + ((l & 1) ? g.pyr_lds_a : g.pyr_lds_b) : nullptr;
        uint8_t* dst_hbm = pyr + V.offset + (size_t)f * V.frame_bytes;
        resize_band(s_pyr, V, b.x, b.y, b.z, b.w, ptab + V.ptab_offset, s_rows + yoff, dst_lds, dst_hbm);
        yoff += b.y - b.x;
        __syncthreads();
    }
}

}  // namespace

int pyr_threads() { return kPyrThreads; }

hipError_t launch_pyramid(const Geom& g, int batch, const int4* bands, const int4* ptab, const int2* ytab,
                          const uint8_t* img0, size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    if (g.nlevels < 2) return hipSuccess;
    hipLaunchKernelGGL(pyramid_kernel, dim3(g.pyr_bands * batch), dim3(kPyrThreads), g.pyr_lds_bytes, stream, g,
                       bands, ptab, ytab, img0, row0, frame0, pyr);
    return hipGetLastError();
}

hipError_t pyramid_set_lds_limit(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace orbgpu
